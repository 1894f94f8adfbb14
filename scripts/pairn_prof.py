"""Driver for rocprofv3 passes on K_pairN: 1024 streams x 480 000 of one shape
(PN_SHAPE="N/H", default 1764/441), a few round trips."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    n, h = (int(v) for v in os.environ.get("PN_SHAPE", "1764/441").split("/"))
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand((1024, 480000), generator=g, device="cuda") * 2 - 1) * 0.5
    plan = pkg.Plan(frame_size=n, hop_size=h)
    y = torch.empty((1024, plan.output_length(480000)), device="cuda")
    for _ in range(4):
        plan.roundtrip(x, y)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

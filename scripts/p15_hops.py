"""Round-trip throughput at several frame/hop shapes (1024 streams x 480 000;
P15_SHAPES="N/H,..." overrides the K_pair15 default list)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [tuple(int(v) for v in sh.split("/")) for sh in os.environ.get("P15_SHAPES", "").split(",") if sh] or \
    [(960, 240), (960, 480), (960, 320), (480, 120), (480, 240)]


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand((1024, 480000), generator=g, device="cuda") * 2 - 1) * 0.5
    for n, h in SHAPES:
        plan = pkg.Plan(frame_size=n, hop_size=h)
        y = torch.empty((1024, plan.output_length(480000)), device="cuda")
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:
            plan.roundtrip(x, y)
            torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(10):
                plan.roundtrip(x, y)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) / 10)
        ms = sorted(ts)[2] * 1e3
        print(json.dumps({"shape": f"{n}/{h}", "ms": round(ms, 4), "Msamples_s": round(1024 * 480000 / ms / 1e3, 1)}))


if __name__ == "__main__":
    main()

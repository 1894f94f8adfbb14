"""Batched round-trip throughput of arbitrary N/H shapes at 1024 streams x 480 000
samples (as scripts/bench_configs.py times them: 200 ms clock warm-up, median of
5 groups of 10 launches).  Usage: python scripts/bench_shapes.py 4096/1024 4096/512 ...
Environment switches apply per process, so A/Bs of two
walkers alternate processes (scripts/ab_env.sh)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    S, T = int(os.environ.get("BS_S", 1024)), 480000
    tag = os.environ.get("BS_TAG", "")
    for shape in sys.argv[1:]:
        N, H = (int(v) for v in shape.split("/"))
        plan = pkg.Plan(frame_size=N, hop_size=H)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
        y = torch.empty((S, plan.output_length(T)), device="cuda")
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:
            plan.roundtrip(x, y)
            torch.cuda.synchronize()
        groups = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                plan.roundtrip(x, y)
            e1.record()
            torch.cuda.synchronize()
            groups.append(e0.elapsed_time(e1) / 10)
        ms = sorted(groups)[2]
        print(json.dumps({"tag": tag, "shape": shape, "streams": S, "ms": round(ms, 4),
                          "Msamples_s": round(S * T / (ms * 1e-3) / 1e6, 1)}), flush=True)
        del x, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

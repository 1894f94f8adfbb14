"""Chunks-per-stream sweep in one process (crlot_plan_set_chunks per setting; the
launch record confirms the chunking each run used).
usage: python scripts/sweep_inproc.py [S T N H] [n1,n2,...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(plan, x, y, torch):
    t_end = time.perf_counter() + 0.15
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
    return sorted(groups)[2]


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    a = sys.argv[1:]
    S, T, N, H = (int(v) for v in a[:4]) if len(a) >= 4 else (1024, 480000, 1024, 256)
    ns = [int(v) for v in a[4].split(",")] if len(a) >= 5 else [0, 4, 8, 12, 15, 16, 20, 24, 32]
    g = torch.Generator(device="cuda").manual_seed(1)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    for pairing in ((True, False) if os.environ.get("SW_BOTH") else (True,)):
        plan = pkg.Plan(frame_size=N, hop_size=H, frame_pairing=pairing)
        y = torch.empty((S, plan.output_length(T)), device="cuda")
        for n in ns:
            plan.set_chunks(n)
            ms = timeit(plan, x, y, torch)
            rec = plan.last_launch()
            print(json.dumps({"pairing": pairing, "chunks": n or "auto", "n_chunks": rec["n_chunks"],
                              "kernels": rec["kernels"], "ms": round(ms, 4),
                              "Msamples_s": round(S * T / ms / 1e3, 1)}), flush=True)
        plan.set_chunks(0)


if __name__ == "__main__":
    main()

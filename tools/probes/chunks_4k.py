"""Probe: config 3 (4096/1024, 1024 x 480000) at forced chunk counts per stream
(Plan.set_chunks; 0 = the chooser), interleaved rounds, median ms."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    n, h = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4096/1024").split("/"))
    S, T = 1024, 480000
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    plan = pkg.Plan(frame_size=n, hop_size=h)
    y = torch.empty((S, plan.output_length(T)), device="cuda")
    knobs = [0, 1, 2, 3, 4, 6]
    times = {k: [] for k in knobs}
    for _ in range(30):
        plan.roundtrip(x, y)
    torch.cuda.synchronize()
    for rnd in range(6):
        for k in knobs[rnd % len(knobs):] + knobs[:rnd % len(knobs)]:
            plan.set_chunks(k)
            plan.roundtrip(x, y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                plan.roundtrip(x, y)
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 5)
    plan.set_chunks(0)
    plan.roundtrip(x, y)
    for k in knobs:
        t = sorted(times[k])[len(times[k]) // 2]
        print(json.dumps({"n": n, "h": h, "chunks": k, "ms": round(t, 4), "Msamples_s": round(S * T / t / 1e3, 1)}))
    print(json.dumps({"auto_launch": plan.last_launch()}))


if __name__ == "__main__":
    main()

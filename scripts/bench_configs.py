"""Throughput of the batched round trip for the BASELINE configs on one GPU
(the headline is bench.py; these are the other shapes): Msamples/s and the
algorithmic HBM fraction (8 B/sample vs 8 TB/s), with the CPU oracle timed
beside each config on the same workload (this host's CPU share, 1 warm-up + 5
timed passes, median: BASELINE.md:51-63; BC_NO_CPU=1 skips it)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [
    ("config2: 256 streams, N=1024 H=256", 256, 480000, 1024, 256, 0),
    ("headline: 1024 streams, N=1024 H=256", 1024, 480000, 1024, 256, 0),
    ("config3: 1024 streams, N=4096 H=1024", 1024, 480000, 4096, 1024, 0),
    ("e2e-harness hop: 1024 streams, N=1024 H=512", 1024, 480000, 1024, 512, 0),
    ("config4 shape batched: 64 ch, N=512 H=128 DROP", 64, 480000, 512, 128, 1),
    ("2048/512: 1024 streams", 1024, 480000, 2048, 512, 0),
    ("any-size 960/240 (20 ms @ 48 kHz): 1024 streams", 1024, 480000, 960, 240, 0),
    ("any-size 480/120 (10 ms @ 48 kHz): 1024 streams", 1024, 480000, 480, 120, 0),
]


def cpu_leg(S, T, N, H, mode, reps=5):
    """The oracle restatement of the reference CPU path on the config's whole
    workload: one warm-up pass, `reps` timed passes, median."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from bench import cpu_share
    threads = cpu_share()
    x = O.synth_streams(S, T, config_id=2)
    O.roundtrip_batch(x, N, H, mode=mode, nthreads=threads, native=True)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        O.roundtrip_batch(x, N, H, mode=mode, nthreads=threads, native=True)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return {"value": round(S * T / dt / 1e6, 2), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "reps": reps, "rep_seconds": [round(t, 3) for t in ts]}


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    only = os.environ.get("BC_ONLY")
    for name, S, T, N, H, mode in CONFIGS:
        if only and only not in name:
            continue
        plan = pkg.Plan(frame_size=N, hop_size=H, boundary_mode=mode)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
        y = torch.empty((S, plan.output_length(T)), device="cuda")
        # warm up for >= 200 ms (clocks ramp), then the median of 5 groups of 10
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:
            plan.roundtrip(x, y)
            torch.cuda.synchronize()
        groups = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                plan.roundtrip(x, y)
            e1.record()
            torch.cuda.synchronize()
            groups.append(e0.elapsed_time(e1) / reps)
        ms = sorted(groups)[len(groups) // 2]
        rate = S * T / (ms * 1e-3)
        rec = plan.last_launch()
        del x, y
        torch.cuda.empty_cache()
        row = {"config": name, "ms": round(ms, 4), "Msamples_s": round(rate / 1e6, 1),
               "hbm_frac_algorithmic": round(8 * rate / 8e12, 4), "kernels": rec["kernels"],
               "n_chunks": rec["n_chunks"]}
        if not os.environ.get("BC_NO_CPU"):
            row["cpu_baseline"] = cpu_leg(S, T, N, H, mode)
            row["gpu_over_cpu"] = round(row["Msamples_s"] / row["cpu_baseline"]["value"], 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

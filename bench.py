"""bench.py -- headline benchmark (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Metric: Msamples/s of the batched STFT -> iSTFT -> OLA round trip at
frame=1024 hop=256 batch=1024 (1024 synthetic mono streams x 480 000 samples
of 48 kHz audio = 10 s each, per GPU), inputs and outputs resident in HBM.
A "step" is one crlot_roundtrip over the whole batch.  N GPUs = N ranks, each
with its own 1024 streams (weak scaling, no data-path collective: the streams
are independent).

Besides the contract fields the JSON line carries
  roofline      the fused kernel's algorithmic HBM bytes (8 B per sample: 4 in,
                4 out) per launch / its average launch time, measured with HIP
                events on the launch stream inside the timed region; traffic =
                PMC HBM bytes per launch from profiles/ (separate rocprofv3 run)
  compute       the same launches priced in FP32 VALU flops
  cpu_baseline  the oracle's C restatement of the reference CPU path (kissfft
                algorithm + scalar-FMA OLA, "kind": "port") timed on this host,
                rank 0 at N=1 only, on a bounded sample of streams.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s STFT->OLA round-trip, frame=1024 hop=256 batch=1024; HBM roofline %"
N_FFT, HOP, STREAMS, T_LEN = 1024, 256, 1024, 480_000
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 vector peak (spec)
BYTES_PER_SAMPLE = 8           # 4 B read + 4 B written


def flop_per_sample(n: int, h: int) -> float:
    """2 x 2.5 N log2 N per frame (rfft + irfft) / H, + ~6 elementwise."""
    import math
    return 2 * 2.5 * n * math.log2(n) / h + 6


def cpu_baseline(n_streams: int = 1024, threads: int = 16):
    """Oracle restatement of the reference CPU path on this host (kind "port")."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    native = False
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True,
                       capture_output=True, timeout=120)
        native = True
    except Exception:
        pass
    threads = max(1, min(threads, os.cpu_count() or 1))
    x = O.synth_streams(n_streams, T_LEN, config_id=2)
    O.roundtrip_batch(x[:threads], N_FFT, HOP, nthreads=threads, native=native)  # warm-up
    t0 = time.perf_counter()
    O.roundtrip_batch(x, N_FFT, HOP, nthreads=threads, native=native)
    dt = time.perf_counter() - t0
    x1 = x[:4]
    t1 = time.perf_counter()
    O.roundtrip_batch(x1, N_FFT, HOP, nthreads=1, native=native)
    dt1 = time.perf_counter() - t1
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": round(n_streams * T_LEN / dt / 1e6, 3),
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_streams} of the 1024 streams x {T_LEN} samples (the N=1 workload), {threads} pthreads, "
                  f"oracle/crlot_oracle.c -O3{' -march=native' if native else ''} "
                  f"(kissfft-algorithm + scalar-FMA OLA restatement), {dt:.2f} s",
        "single_thread_value": round(4 * T_LEN / dt1 / 1e6, 3),
        "cpu_model": cpu_model,
    }


def load_pmc_traffic():
    """HBM bytes per launch from the newest profiles/*pmc*.json (rocprofv3 --pmc run)."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if os.path.isdir(pdir):
        for f in sorted(os.listdir(pdir)):
            if f.endswith(".json") and "pmc" in f and not f.startswith("_"):
                try:
                    d = json.load(open(os.path.join(pdir, f)))
                except Exception:
                    continue
                if d.get("workload_key") == f"{STREAMS}x{T_LEN}_N{N_FFT}_H{HOP}":
                    best = d
    return None if best is None else best.get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50)  # ~130 ms: lets the clocks ramp
    ap.add_argument("--streams", type=int, default=STREAMS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    from __graft_entry__ import load_pkg, load_dist

    D = load_dist()
    _, world, local = D.env_rank_world()
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    rank, world = D.init("nccl", dev)

    pkg = load_pkg()
    plan = pkg.Plan(frame_size=N_FFT, hop_size=HOP, device=dev.index)
    S, T = args.streams, T_LEN
    g = torch.Generator(device=dev).manual_seed(0xC0FFEE + rank)
    x = (torch.rand((S, T), generator=g, device=dev) * 2.0 - 1.0) * 0.5
    L = plan.output_length(T)
    y = torch.empty((S, L), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        plan.roundtrip(x, y)
    torch.cuda.synchronize(dev)

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    D.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        plan.roundtrip(x, y)
        ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    D.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    elapsed_max = D.max_over_ranks(elapsed, dev)

    samples_step_rank = S * T
    total_samples = samples_step_rank * world * args.steps
    value = total_samples / elapsed_max / 1e6
    achieved_gbs = BYTES_PER_SAMPLE * samples_step_rank / (kern_ms * 1e-3) / 1e9
    fps = flop_per_sample(N_FFT, HOP)
    achieved_tf = fps * samples_step_rank / (kern_ms * 1e-3) / 1e12
    traffic = load_pmc_traffic()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline()
        except Exception as e:  # reported, never fatal to the GPU number
            cpu = {"value": None, "unit": "Msamples/s", "cores": 0, "kind": "port",
                   "sample": f"failed: {e}"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform[-0.5,0.5) float32 streams generated on device, HBM-resident",
            "config": {
                "workload": f"{S} mono streams x {T} samples (48 kHz, 10 s) per GPU, "
                            f"N={N_FFT} H={HOP} symmetric Hann, ZERO_PAD framing, "
                            "frame*w -> rfft -> irfft -> OLA(window inside) -> /max(norm,eps)",
                "streams_per_gpu": S,
                "samples_per_stream": T,
                "frame": N_FFT,
                "hop": HOP,
                "global_batch": S * world,
                "parallelism": f"streams sharded over {world} rank(s), no collective",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel_ms": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": BYTES_PER_SAMPLE * samples_step_rank,
            },
            "compute": {
                "flop_per_sample": round(fps, 1),
                "achieved_tflops": round(achieved_tf, 2),
                "peak_tflops": VALU_PEAK_TFLOPS,
                "frac": round(achieved_tf / VALU_PEAK_TFLOPS, 4),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    D.finalize()


if __name__ == "__main__":
    main()

"""BASELINE config 1 (CPU plumbing case) end to end on the product path:
assets/oboe.wav (tests/golden/oboe.wav, the reference's own asset) -> WavReader
-> mono mixdown (main/main.cc:155-160) -> N=1024 / H=256 symmetric Hann round
trip -> WavWriter (16-bit).  The round trip runs on the GPU when one is present
and always on the CPU oracle (the reference path restated, checker only), both
timed; prints one JSON line and writes gpurun_out/oboe_roundtrip.wav.

    python scripts/config1_wav.py [--out PATH]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "oboe_roundtrip.wav"))
    args = ap.parse_args()
    from __graft_entry__ import load_pkg
    import oracle as O  # checker / CPU timing only
    pkg = load_pkg()
    x, sr = pkg.load_wav_mono(os.path.join(ROOT, "tests", "golden", "oboe.wav"))
    n, h = 1024, 256
    t0 = time.perf_counter()
    ref = O.roundtrip(x, n, h)
    cpu_s = time.perf_counter() - t0
    res = {"config": "config1: oboe.wav mono, N=1024 H=256 Hann", "samples": int(x.size),
           "sample_rate": sr, "cpu_oracle_ms": round(cpu_s * 1e3, 3),
           "cpu_oracle_msamples_s": round(x.size / cpu_s / 1e6, 2)}
    y = ref
    try:
        import torch
        gpu = torch.cuda.is_available()
    except Exception:
        gpu = False
    if gpu:
        plan = pkg.Plan(frame_size=n, hop_size=h)
        xd = torch.from_numpy(x[None]).cuda()
        out = plan.roundtrip(xd)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            plan.roundtrip(xd, out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        y = out[0].cpu().numpy()
        d = y.astype(np.float64) - ref
        res.update(gpu_ms=round(ms, 4), gpu_msamples_s=round(x.size / ms / 1e3, 1),
                   rel_l2_vs_oracle=float(np.linalg.norm(d) / np.linalg.norm(ref)),
                   max_abs_vs_oracle=float(np.max(np.abs(d))))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    w = pkg.WavWriter()
    assert w.open(args.out, 1, sr, 16)
    w.write(np.clip(y[:x.size], -1, 1))
    w.close()
    res["wrote"] = os.path.relpath(args.out, ROOT)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

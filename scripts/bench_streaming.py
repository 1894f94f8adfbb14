"""BASELINE config 4: 64-channel 48 kHz streaming, N=512 H=128, DROP framing,
per-hop push of 64 x 128 samples for 10 s of audio (3750 hops).  Reports p50/p99
per-hop latency (host wall around push + synchronize, and device time from HIP
events) and the sustained rate, next to the oracle doing the same per-hop work on
one CPU core.  Latency-bound and cache-resident: no HBM roofline claim."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

C_, N, H, SR, SECONDS = 64, 512, 128, 48000, 10
HOPS = SR * SECONDS // H


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    plan = pkg.Plan(frame_size=N, hop_size=H, boundary_mode=pkg.DROP)
    st = pkg.Stream(plan, C_, interleaved=True)
    g = torch.Generator(device="cuda").manual_seed(4)
    x = ((torch.rand((HOPS, H, C_), generator=g, device="cuda") * 2 - 1) * 0.5).contiguous()
    out = torch.empty((H, C_), device="cuda")
    for q in range(16):  # warm-up
        st.push_hop(x[q], out)
    torch.cuda.synchronize()
    st.reset()
    wall, devt = [], []
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_all = time.perf_counter()
    for q in range(HOPS):
        t0 = time.perf_counter()
        ev0.record()
        st.push_hop(x[q], out)
        ev1.record()
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        devt.append(ev0.elapsed_time(ev1) * 1e-3)
    t_all = time.perf_counter() - t_all
    # back-to-back (no per-hop sync): sustained device throughput
    torch.cuda.synchronize()
    st.reset()
    t0 = time.perf_counter()
    for q in range(HOPS):
        st.push_hop(x[q], out)
    torch.cuda.synchronize()
    t_b2b = time.perf_counter() - t0

    # CPU: the oracle doing the same per-hop streaming work for one channel on one core,
    # scaled to 64 channels (the channels are independent)
    import oracle as O
    xs = O.synth(HOPS * H // 10, 9)
    t0 = time.perf_counter()
    O.roundtrip(xs, N, H, mode=O.DROP)
    cpu_per_hop_1ch = (time.perf_counter() - t0) / (xs.size // H)
    w = np.array(wall) * 1e6
    d = np.array(devt) * 1e6
    print(json.dumps({
        "config": "64ch x 48kHz streaming, N=512 H=128 DROP, per-hop push, 10 s (3750 hops)",
        "hop_latency_us_wall": {"p50": round(float(np.percentile(w, 50)), 2),
                                "p99": round(float(np.percentile(w, 99)), 2),
                                "max": round(float(w.max()), 2)},
        "hop_latency_us_device": {"p50": round(float(np.percentile(d, 50)), 2),
                                  "p99": round(float(np.percentile(d, 99)), 2)},
        "hop_budget_us_realtime": round(H / SR * 1e6, 1),
        "sustained_Msamples_s_synced": round(HOPS * H * C_ / t_all / 1e6, 2),
        "sustained_Msamples_s_back_to_back": round(HOPS * H * C_ / t_b2b / 1e6, 2),
        "realtime_factor_back_to_back": round(SECONDS / t_b2b, 1),
        "cpu_oracle_1core_us_per_hop_64ch": round(cpu_per_hop_1ch * C_ * 1e6, 1),
    }))


if __name__ == "__main__":
    main()

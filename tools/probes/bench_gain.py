"""Throughput of the round trip with a spectral gain (the §8f spectral hook) next to
the plain plan, headline shape (1024 streams x 480 000, N=1024 H=256)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    S, T = 1024, 480000
    N, H = int(os.environ.get("BG_N", 1024)), int(os.environ.get("BG_H", 256))
    g = torch.Generator(device="cuda").manual_seed(5)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    for label, gain in (("no gain", None), ("spectral gain", np.linspace(0.5, 1.5, N // 2 + 1).astype(np.float32))):
        plan = pkg.Plan(frame_size=N, hop_size=H)
        if gain is not None:
            plan.set_spectral_gain(gain)
        y = torch.empty((S, plan.output_length(T)), device="cuda")
        for _ in range(20):
            plan.roundtrip(x, y)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                plan.roundtrip(x, y)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        ms = sorted(ts)[2]
        print(json.dumps({"case": label, "ms": round(ms, 4), "Msamples_s": round(S * T / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()

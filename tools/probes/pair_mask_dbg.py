"""Probe: K_pair_mask vs K_pair (mask of ones) and vs the per-frame masked walk,
per stream and OLA block (max abs difference, first blocks that differ), on plain
and special input.  usage: pair_mask_dbg.py [N/H]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    from __graft_entry__ import load_pkg
    import oracle as O
    from test_gpu_stft import special
    pkg = load_pkg()
    n, h = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1024/256").split("/"))
    S = 4
    T = 29 * n + 17
    plan = pkg.Plan(frame_size=n, hop_size=h)
    F = plan.frame_count(T)
    for name, x in (("plain", O.synth_streams(S, T, config_id=68)), ("special", special(O.synth_streams(S, T, config_id=68)))):
        xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
        plan.set_spectral_mask(None)
        y0 = plan.roundtrip(xd).cpu().numpy()
        k0 = plan.last_launch()["kernels"]
        plan.set_spectral_mask(torch.ones((F, n // 2 + 1), device="cuda"))
        y1 = plan.roundtrip(xd).cpu().numpy()
        k1 = plan.last_launch()["kernels"]
        plan.set_spectral_mask(None)
        d = np.abs(y1.astype(np.float64) - y0).reshape(S, F, h).max(axis=2)
        for s in range(S):
            bad = np.nonzero(d[s] > 0)[0]
            print(name, k0, k1, "stream", s, "max", float(d[s].max()), "scale", float(np.nanmax(np.abs(y0[s]))),
                  "blocks", bad[:12].tolist(), len(bad), flush=True)


if __name__ == "__main__":
    main()

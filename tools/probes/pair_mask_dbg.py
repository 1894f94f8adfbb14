"""Probe: K_pair_mask vs the per-frame masked walk on plain / special inputs,
per stream and per frame (rel error), to localise a mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    n, h, S = 1024, 256, 3
    T = 13 * n + 31
    rng = np.random.default_rng(1)
    x = rng.uniform(-0.5, 0.5, (S, T)).astype(np.float32)
    plan = pkg.Plan(frame_size=n, hop_size=h)
    F = plan.frame_count(T)
    xd = torch.from_numpy(x).cuda()
    for name, m in (("ones", np.ones((F, n // 2 + 1), np.float32)),
                    ("const2", np.full((F, n // 2 + 1), 2.0, np.float32)),
                    ("rowvar", np.repeat(np.linspace(0.1, 1.0, F, dtype=np.float32)[:, None], n // 2 + 1, 1)),
                    ("binvar", np.repeat(np.linspace(0.1, 1.0, n // 2 + 1, dtype=np.float32)[None], F, 0)),
                    ("rand", rng.uniform(0, 1, (F, n // 2 + 1)).astype(np.float32))):
        plan.set_spectral_mask(torch.from_numpy(m).cuda())
        plan.set_frame_pairing(True)
        y = plan.roundtrip(xd).cpu().numpy()
        k = plan.last_launch()["kernels"]
        plan.set_frame_pairing(False)
        yf = plan.roundtrip(xd).cpu().numpy()
        d = np.abs(y - yf).reshape(S, F, h).max(axis=(0, 2))
        bad = np.nonzero(d > 1e-5)[0]
        print(name, k, "max", float(np.abs(y - yf).max()), "bad blocks", bad[:20].tolist(), len(bad), flush=True)
    plan.set_spectral_mask(None)


if __name__ == "__main__":
    main()

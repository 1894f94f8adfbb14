"""Host-buffer streaming latency per hop (StreamRT.push_hop, wall p50/p99) at
the resident shapes and at launch-mode shapes (20 / 10 ms frames at 48 kHz),
stereo and 64 channels: one JSON line per shape."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (device init as the package expects)
    from __graft_entry__ import load_pkg
    pkg = load_pkg()
    for n, h, C in ((512, 128, 64), (1024, 512, 2), (960, 480, 2), (960, 240, 2), (480, 240, 2), (960, 480, 64)):
        plan = pkg.Plan(frame_size=n, hop_size=h, boundary_mode=pkg.DROP, frame_pairing=False)
        st = pkg.StreamRT(plan, C, interleaved=True)
        x = (np.random.default_rng(1).random((h, C), dtype=np.float32) - 0.5)
        for _ in range(50):
            st.push_hop(x)
        ts = []
        for _ in range(2000):
            t0 = time.perf_counter()
            st.push_hop(x)
            ts.append((time.perf_counter() - t0) * 1e6)
        resident = bool(st.info()["running"])
        st.close()
        ts.sort()
        print(json.dumps({"frame": n, "hop": h, "channels": C, "mode": "resident" if resident else "launch",
                          "wall_us_p50": round(ts[len(ts) // 2], 2), "wall_us_p99": round(ts[int(len(ts) * 0.99)], 2),
                          "hop_ms_realtime": round(1e3 * h / 48000, 3)}), flush=True)


if __name__ == "__main__":
    main()

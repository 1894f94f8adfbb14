"""Per-wave timeline of K_pair from a CRLOT_PAIR_TRACE build (variants/libcrlot_dsp_trace.so):
wave start/end (100 MHz s_memrealtime) and hardware ids; prints the duration spread,
the mean resident waves per SIMD and how long each CU idles between its workgroups."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

lib = os.path.join(ROOT, "crlot-dsp_amd", "variants", "libcrlot_dsp_trace.so")
os.environ["CRLOT_LIB"] = lib
from __graft_entry__ import load_pkg  # noqa: E402

pkg = load_pkg()
L = pkg.lib()
S, T = int(os.environ.get("TL_S", 1024)), 480000
plan = pkg.Plan(frame_size=1024, hop_size=256)
g = torch.Generator(device="cuda").manual_seed(3)
x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
y = torch.empty((S, plan.output_length(T)), device="cuda")
for _ in range(30):
    plan.roundtrip(x, y)
torch.cuda.synchronize()
buf = np.zeros((1 << 16, 4), np.uint32)
L.crlot_debug_pair_trace.argtypes = [C.c_void_p, C.c_int64]
assert L.crlot_debug_pair_trace(buf.ctypes.data, buf.nbytes) == 0
n = int(np.count_nonzero(buf[:, 1]))
t = buf[:n].astype(np.int64)
t0 = t[:, 0].min()
st, en = t[:, 0] - t0, t[:, 1] - t0
dur = (en - st) / 100.0  # us
hw, xcc = t[:, 2], t[:, 3]
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
cuid = (xcc & 15) * 1000 + se * 100 + cu
span = (en.max()) / 100.0
out = {"waves": n, "kernel_span_us": span, "dur_us_min": float(dur.min()), "dur_us_med": float(np.median(dur)),
       "dur_us_max": float(dur.max()), "dur_us_p10": float(np.percentile(dur, 10)), "dur_us_p90": float(np.percentile(dur, 90)),
       "mean_resident_waves_per_simd": float(dur.sum() / span / (len(np.unique(cuid)) * 4)),
       "cus_seen": int(len(np.unique(cuid))), "start_us_max_first_round": None}
# per CU: workgroups in order of start; idle gap between last end of WG i and first start of WG i+1
gaps, wg_spread = [], []
for c in np.unique(cuid):
    m = cuid == c
    s_, e_ = st[m], en[m]
    order = np.argsort(s_)
    s_, e_ = s_[order], e_[order]
    # group waves into workgroups by start time clusters (16 per WG)
    for i in range(0, len(s_), 16):
        grp_e = e_[i:i + 16]
        wg_spread.append((grp_e.max() - grp_e.min()) / 100.0)
        if i + 16 < len(s_):
            gaps.append((s_[i + 16:i + 32].min() - grp_e.max()) / 100.0)
out["wg_end_spread_us_med"] = float(np.median(wg_spread))
out["wg_end_spread_us_max"] = float(np.max(wg_spread))
out["gap_between_wgs_us_med"] = float(np.median(gaps)) if gaps else None
out["cu_finish_us_min"] = float(min(en[cuid == c].max() for c in np.unique(cuid)) / 100.0)
out["cu_finish_us_med"] = float(np.median([en[cuid == c].max() for c in np.unique(cuid)]) / 100.0)
# simd-age effect: duration by rank of start within its SIMD
print(json.dumps(out, indent=1))
hist = np.histogram(dur, bins=12)
print("duration histogram (us):", [(round(float(a), 1), int(b)) for a, b in zip(hist[1], hist[0])])

"""Cycles per pair by loop phase of K_pair, from a CRLOT_PAIR_PHASES build
(variants/libcrlot_dsp_phases.so; s_memtime stamps, which themselves cost cycles)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

os.environ["CRLOT_LIB"] = os.path.join(ROOT, "crlot-dsp_amd", "variants", "libcrlot_dsp_phases.so")
from __graft_entry__ import load_pkg  # noqa: E402

pkg = load_pkg()
L = pkg.lib()
S, T = 1024, 480000
plan = pkg.Plan(frame_size=1024, hop_size=256)
x = (torch.rand((S, T), device="cuda") * 2 - 1) * 0.5
y = torch.empty((S, plan.output_length(T)), device="cuda")
for _ in range(20):
    plan.roundtrip(x, y)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
plan.roundtrip(x, y)
e1.record()
torch.cuda.synchronize()
print("kernel ms (instrumented)", e0.elapsed_time(e1))
buf = np.zeros((1 << 16, 8), np.uint32)
L.crlot_debug_pair_phases.argtypes = [C.c_void_p, C.c_int64]
assert L.crlot_debug_pair_phases(buf.ctypes.data, buf.nbytes) == 0
b = buf[buf[:, 7] == 1].astype(np.float64)
pairs = b[:, 6]
names = ["tail+loop (hop check, shift, wait x)", "prefetch issue + build v", "forward fft", "gain + inverse fft",
         "den loads + OLA + 2 emits", "epilogue"]
tot = b[:, :6].sum(axis=1)
print("waves", len(b), "pairs/wave", pairs.mean(), "cycles/pair/wave", (tot / pairs).mean())
for i, n in enumerate(names):
    print(f"{n:40s} {np.mean(b[:, i] / pairs):9.1f} cycles/pair  ({100 * b[:, i].sum() / tot.sum():5.1f} %)")

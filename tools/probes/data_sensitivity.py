"""Does the round trip's speed depend on the sample values?  (A power/clock-limited
kernel runs faster on low-toggle data.)  Times the headline workload on uniform
random, zero and constant input, and reports the GPU clock from GRBM-free
estimates (HIP events only)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from __graft_entry__ import load_pkg  # noqa: E402

pkg = load_pkg()
S, T = 1024, 480000
plan = pkg.Plan(frame_size=1024, hop_size=256)
g = torch.Generator(device="cuda").manual_seed(1)
inputs = {
    "uniform": (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5,
    "zeros": torch.zeros((S, T), device="cuda"),
    "const": torch.full((S, T), 0.25, device="cuda"),
    "sine": torch.sin(torch.arange(T, device="cuda", dtype=torch.float32) * 0.01).repeat(S, 1) * 0.5,
}
y = torch.empty((S, plan.output_length(T)), device="cuda")
for rnd in range(2):
    for name, x in inputs.items():
        t_end = time.perf_counter() + 0.3
        while time.perf_counter() < t_end:
            plan.roundtrip(x, y)
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            plan.roundtrip(x, y)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"round": rnd, "input": name, "ms": round(ms, 4), "Msamples_s": round(S * T / ms / 1e3, 1)}), flush=True)

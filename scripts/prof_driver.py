"""Minimal driver for rocprofv3 PMC passes: run the headline round trip a few
times (1024 streams x 480000, N=1024 H=256) with nothing else on the GPU."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--streams", type=int, default=1024)
ap.add_argument("--T", type=int, default=480000)
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--h", type=int, default=256)
ap.add_argument("--data", default="uniform", choices=["uniform", "zeros"])
args = ap.parse_args()

import torch  # noqa: E402
from __graft_entry__ import load_pkg  # noqa: E402

pkg = load_pkg()
plan = pkg.Plan(frame_size=args.n, hop_size=args.h)
g = torch.Generator(device="cuda").manual_seed(7)
x = (torch.rand((args.streams, args.T), generator=g, device="cuda") * 2 - 1) * 0.5
if args.data == "zeros":
    x.zero_()
y = torch.empty((args.streams, plan.output_length(args.T)), device="cuda")
for _ in range(args.reps):
    plan.roundtrip(x, y)
torch.cuda.synchronize()
print("prof driver done", flush=True)

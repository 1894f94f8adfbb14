"""Diagnostics: which K_pair chunks the paired-only walker hands to the fix-up
walker, found by running with CRLOT_PAIR_NOFIX=1 (child process) and diffing
against the full result per output block."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S, T, N, H = int(os.environ.get("PF_S", 64)), 480000, 1024, 256

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, ROOT)
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_pkg()
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.rand((S, T), generator=g, device="cuda") * 2 - 1) * 0.5
    y = pkg.Plan(frame_size=N, hop_size=H).roundtrip(x)
    torch.cuda.synchronize()
    torch.save(y.cpu(), sys.argv[2])
    sys.exit(0)

import torch  # noqa: E402
outs = []
for nofix in ("0", "1"):
    f = f"/tmp/pf_{nofix}.pt"
    env = dict(os.environ, CRLOT_PAIR_NOFIX=nofix)
    subprocess.run([sys.executable, __file__, "child", f], env=env, check=True)
    outs.append(torch.load(f, weights_only=True))
a, b = outs
F = a.shape[1] // H
diff = (a.view(S, F, H) != b.view(S, F, H)).any(dim=2)
print(f"blocks differing: {int(diff.sum())} of {S * F} ({float(diff.float().mean()):.4f})")
per_stream = diff.any(dim=1).sum()
first = [int(diff[s].nonzero()[0]) if diff[s].any() else -1 for s in range(min(S, 8))]
print("streams with any:", int(per_stream), "first differing block per stream:", first)
cols = diff.any(dim=0).nonzero().flatten().tolist()
print("block indices differing in any stream (first 40):", cols[:40], "count", len(cols))

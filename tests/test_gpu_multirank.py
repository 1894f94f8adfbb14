"""Multi-rank path on the device (BASELINE config 5 in small):
two ranks (gloo control plane) share the one GPU of the box, each runs the HIP
library on its dist.stream_range block, and the assembled output equals a
single-process run bit for bit (the round trip's bits do not depend on the
batch a stream is in).  Also runs bench.py --gpus 2 through its own launcher."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from __graft_entry__ import load_pkg, load_dist
import torch
D = load_dist()
_, world, local = D.env_rank_world()
dev = torch.device("cuda", D.device_for(local, torch.cuda.device_count()))
torch.cuda.set_device(dev)
rank, world = D.init("gloo")
import oracle as O
S_total, T = 10, 48000
lo, hi = D.stream_range(S_total, world, rank)
x = O.synth_streams(S_total, T, config_id=5)[lo:hi]
pkg = load_pkg()
plan = pkg.Plan(frame_size=1024, hop_size=256, device=dev.index)
D.barrier()
y = plan.roundtrip(torch.from_numpy(x).to(dev))
torch.cuda.synchronize(dev)
D.barrier()
np.save(os.path.join(OUT, f"y_{rank}.npy"), y.cpu().numpy())
json.dump({"rank": rank, "lo": lo, "hi": hi, "device": dev.index,
           "mx": D.max_over_ranks(float(rank))}, open(os.path.join(OUT, f"r_{rank}.json"), "w"))
D.finalize()
'''


@pytest.mark.gpu
def test_two_ranks_one_gpu_hip_bit_exact(tmp_path, torch_cuda, pkg, oracle):
    torch = torch_cuda
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\n" + WORKER)
    sys.path.insert(0, ROOT)
    from __graft_entry__ import load_dist
    D = load_dist()
    assert D.launch(2, [str(script)], timeout=240) == 0
    rs = [json.load(open(tmp_path / f"r_{r}.json")) for r in range(2)]
    assert [(r["lo"], r["hi"]) for r in rs] == [(0, 5), (5, 10)]
    assert all(r["mx"] == 1.0 for r in rs)
    y = np.concatenate([np.load(tmp_path / f"y_{r}.npy") for r in range(2)])
    x = oracle.synth_streams(10, 48000, config_id=5)
    plan = pkg.Plan(frame_size=1024, hop_size=256)
    y1 = plan.roundtrip(torch.from_numpy(x).to("cuda:0")).cpu().numpy()
    assert np.array_equal(y, y1)
    ref = oracle.roundtrip_batch(x, 1024, 256, nthreads=4)
    assert np.linalg.norm(y - ref) <= 1e-6 * np.linalg.norm(ref)


@pytest.mark.gpu
def test_bench_launches_its_own_ranks(torch_cuda):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--streams", "8", "--strong-streams", "16", "--strong-steps", "2",
           "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["ranks"] == 2 and out["config"]["global_batch"] == 16
    assert out["n_gpus"] == min(2, torch_cuda.cuda.device_count())  # distinct devices, not ranks
    assert out["value"] > 0 and out["strong_scaling"]["value"] > 0
    assert out["strong_scaling"]["streams_per_rank"] == [[0, 8], [8, 16]]


CONFIG5_WORKER = r'''
import os, sys, json
import numpy as np
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from __graft_entry__ import load_pkg, load_dist
import torch
D = load_dist()
_, world, local = D.env_rank_world()
dev = torch.device("cuda", D.device_for(local, torch.cuda.device_count()))
torch.cuda.set_device(dev)
rank, world = D.init("gloo")
import oracle as O
lo, hi = D.stream_range(S_TOTAL, world, rank)
x = O.synth_streams(hi - lo, T, config_id=55, first_stream=lo)
pkg = load_pkg()
plan = pkg.Plan(frame_size=1024, hop_size=256, device=dev.index)
D.barrier()
y = plan.roundtrip(torch.from_numpy(x).to(dev))
torch.cuda.synchronize(dev)
D.barrier()
np.save(os.path.join(OUT, f"y_{rank}.npy"), y.cpu().numpy())
json.dump({"rank": rank, "lo": lo, "hi": hi, "mx": D.max_over_ranks(float(rank))},
          open(os.path.join(OUT, f"r_{rank}.json"), "w"))
D.finalize()
'''


@pytest.mark.gpu
def test_config5_8192_streams_over_8_ranks(tmp_path, torch_cuda, pkg, oracle):
    """BASELINE config 5 at its stream count: 8192 independent streams sharded over
    8 ranks (dist.stream_range, no data-path collective; the ranks share this
    box's one GPU, gloo control plane) with short T.  The assembled output equals
    one process's bit for bit; one stream of every shard matches the oracle."""
    torch = torch_cuda
    S_total, T, world = 8192, 4800, 8
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\nS_TOTAL = {S_total}\nT = {T}\n"
                      + CONFIG5_WORKER)
    sys.path.insert(0, ROOT)
    from __graft_entry__ import load_dist
    D = load_dist()
    assert D.launch(world, [str(script)], timeout=300) == 0
    rs = [json.load(open(tmp_path / f"r_{r}.json")) for r in range(world)]
    assert [(r["lo"], r["hi"]) for r in rs] == [(1024 * r, 1024 * (r + 1)) for r in range(world)]
    assert all(r["mx"] == world - 1 for r in rs)
    y = np.concatenate([np.load(tmp_path / f"y_{r}.npy") for r in range(world)])
    x = oracle.synth_streams(S_total, T, config_id=55)
    plan = pkg.Plan(frame_size=1024, hop_size=256)
    y1 = plan.roundtrip(torch.from_numpy(x).to("cuda:0")).cpu().numpy()
    assert y.shape == y1.shape == (S_total, plan.output_length(T))
    assert np.array_equal(y.view(np.uint32), y1.view(np.uint32))
    for s in [1024 * r + (r * 131) % 1024 for r in range(world)]:
        ref = oracle.roundtrip(x[s], 1024, 256)
        assert np.linalg.norm(y[s] - ref) <= 1e-6 * np.linalg.norm(ref), s

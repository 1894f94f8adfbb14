"""world_size-2 coverage of the multi-rank path on CPU (gloo): stream sharding
covers every stream exactly once, per-rank results equal a single-process run,
and the timing reduction is the max over ranks.  The per-rank compute here is
the oracle (CPU), standing in for the device kernel, which the GPU tests cover."""
import os
import socket
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r'''
import os, sys, json, time
import numpy as np
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import importlib.util
spec = importlib.util.spec_from_file_location("crlot_dist", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
D = importlib.util.module_from_spec(spec); spec.loader.exec_module(D)
import oracle as O
rank, world = D.init("gloo")
S_total, T = 6, 5000
lo, hi = D.stream_range(S_total, world, rank)
x = O.synth_streams(S_total, T, config_id=5)[lo:hi]
D.barrier()
t0 = time.perf_counter()
y = O.roundtrip_batch(x, 1024, 256)
dt = time.perf_counter() - t0 + 0.05 * rank   # make ranks differ
D.barrier()
mx = D.max_over_ranks(dt)
np.save(os.path.join(OUT, f"y_{rank}.npy"), y)
json.dump({"rank": rank, "lo": lo, "hi": hi, "dt": dt, "max": mx}, open(os.path.join(OUT, f"r_{rank}.json"), "w"))
D.finalize()
'''


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_sharding_gloo(tmp_path, oracle):
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\n" + WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="2")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=e))
    for p in procs:
        assert p.wait(timeout=300) == 0
    import json
    rs = [json.load(open(tmp_path / f"r_{r}.json")) for r in range(2)]
    assert (rs[0]["lo"], rs[0]["hi"], rs[1]["lo"], rs[1]["hi"]) == (0, 3, 3, 6)
    assert rs[0]["max"] == rs[1]["max"] == max(r["dt"] for r in rs)
    y = np.concatenate([np.load(tmp_path / f"y_{r}.npy") for r in range(2)])
    x = oracle.synth_streams(6, 5000, config_id=5)
    ref = oracle.roundtrip_batch(x, 1024, 256)
    assert np.array_equal(y, ref)


def test_stream_range_partitions():
    import importlib.util
    spec = importlib.util.spec_from_file_location("crlot_dist", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    for total in (1, 7, 1024, 8192):
        for world in (1, 2, 3, 4, 8):
            ranges = [D.stream_range(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def _load_dist():
    import importlib.util
    spec = importlib.util.spec_from_file_location("crlot_dist_t", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    return D


def test_nccl_init_arguments_and_reduce_device(monkeypatch):
    """The RCCL control-plane path without RCCL: init("nccl", dev) hands the rank's
    device to init_process_group (device_id), gloo hands nothing; the max-over-ranks
    reduction runs on the device under nccl and on the host under gloo; a
    single-rank job never initialises a process group."""
    import torch
    import torch.distributed as dist
    D = _load_dist()
    calls = []
    monkeypatch.setattr(dist, "is_initialized", lambda: bool(calls))
    monkeypatch.setattr(dist, "init_process_group", lambda backend, **kw: calls.append((backend, kw)))
    dev = torch.device("cuda", 3)
    assert D.init_kwargs("nccl", dev) == {"device_id": dev}
    assert D.init_kwargs("nccl", None) == {}
    assert D.init_kwargs("gloo", dev) == {}
    try:
        D.init_kwargs("mpi", dev)
        raise AssertionError("unknown backend accepted")
    except ValueError:
        pass
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    assert D.init("nccl", dev) == (0, 1) and calls == []
    assert D.reduce_device(dev) == dev  # backend recorded even for one rank
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "5")
    assert D.init("nccl", dev) == (5, 8)
    import datetime
    assert calls == [("nccl", {"device_id": dev, "timeout": datetime.timedelta(seconds=D.INIT_TIMEOUT_S)})]
    assert D.reduce_device(dev) == dev and D.reduce_device(None) == "cpu"
    D.init("gloo", dev)  # already initialised: no second group
    assert len(calls) == 1 and D.reduce_device(dev) == "cpu"
    # max_over_ranks: the all_reduce sees a tensor on the chosen device
    seen = []
    monkeypatch.setattr(dist, "get_world_size", lambda: 8)
    monkeypatch.setattr(dist, "all_reduce", lambda t, op=None: seen.append((t.device.type, op)))
    assert D.max_over_ranks(1.5, None) == 1.5
    assert seen == [("cpu", dist.ReduceOp.MAX)]


FAILER = r'''
import os, sys, time
import importlib.util
spec = importlib.util.spec_from_file_location("crlot_dist", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
D = importlib.util.module_from_spec(spec); spec.loader.exec_module(D)
rank, world = D.init("gloo", timeout_s=600)
if rank == 1:
    sys.exit(3)  # dies before the barrier
D.barrier()      # rank 0 would wait here for the dead rank
obs = D.observed_world()
D.finalize()
'''

OBSERVER = r'''
import os, sys, json
import importlib.util
spec = importlib.util.spec_from_file_location("crlot_dist", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
D = importlib.util.module_from_spec(spec); spec.loader.exec_module(D)
rank, world = D.init("gloo")
obs = D.observed_world(rank % 2)   # stand-in device ordinals: two distinct "devices"
json.dump(obs, open(os.path.join(OUT, f"obs_{rank}.json"), "w"))
D.finalize()
'''


def _load_dist():
    import importlib.util
    spec = importlib.util.spec_from_file_location("crlot_dist_t", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
    D = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(D)
    return D


def test_launch_fails_fast_when_a_rank_dies(tmp_path):
    """dist.launch polls every rank: rank 1 exiting with 3 before the barrier
    stops rank 0 (blocked in the barrier) and the launcher returns 3 within
    seconds, not after the collective timeout."""
    import time
    D = _load_dist()
    script = tmp_path / "failer.py"
    script.write_text(f"ROOT = {ROOT!r}\n" + FAILER)
    t0 = time.monotonic()
    rc = D.launch(2, [str(script)], timeout=120)
    dt = time.monotonic() - t0
    assert rc == 3 and dt < 10, (rc, dt)


def test_launch_timeout_returns_124(tmp_path):
    D = _load_dist()
    script = tmp_path / "sleeper.py"
    script.write_text("import time\ntime.sleep(60)\n")
    assert D.launch(2, [str(script)], timeout=1.0) == 124


def test_observed_world_counts_ranks_and_devices(tmp_path):
    """observed_world all-gathers each rank's device id: the bench line's record
    of what the process group really held (world size, distinct devices)."""
    import json
    D = _load_dist()
    script = tmp_path / "obs.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\n" + OBSERVER)
    assert D.launch(2, [str(script)], timeout=120) == 0
    for r in range(2):
        o = json.load(open(tmp_path / f"obs_{r}.json"))
        assert o["world"] == 2 and o["backend"] == "gloo" and o["devices"] == 2, o
        assert o["device_keys"] == [0, 1], o


SLOW_WORKER = r'''
import os, sys, json, time
import importlib.util
spec = importlib.util.spec_from_file_location("crlot_dist", os.path.join(ROOT, "crlot-dsp_amd", "dist.py"))
D = importlib.util.module_from_spec(spec); spec.loader.exec_module(D)
rank, world = D.init("gloo")
D.barrier()
t0 = time.perf_counter()
time.sleep(0.2 * (3.0 if rank == SLOW else 1.0))   # rank SLOW is 3x slower
own_ms = (time.perf_counter() - t0) * 1e3
D.barrier()
per = D.gather_over_ranks([own_ms * 0.9, own_ms])   # (kernel ms, wall ms) as bench.py reports them
rep = D.rank_report([p[0] for p in per], [p[1] for p in per], [100 + r for r in range(world)])
json.dump(rep, open(os.path.join(OUT, f"rep_{rank}.json"), "w"))
D.finalize()
'''


def test_slow_rank_is_named_gloo(tmp_path):
    """bench.py's ranks_report (dist.rank_report over an all-gather): with one of
    three ranks made 3x slower, every rank's report names it as the slowest and as
    a straggler, with its device key and times."""
    import json
    world, slow = 3, 1
    script = tmp_path / "worker.py"
    script.write_text(f"ROOT = {ROOT!r}\nOUT = {str(tmp_path)!r}\nSLOW = {slow}\n" + SLOW_WORKER)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(world)]
    for p in procs:
        assert p.wait(timeout=300) == 0
    reps = [json.load(open(tmp_path / f"rep_{r}.json")) for r in range(world)]
    assert all(r == reps[0] for r in reps)
    rep = reps[0]
    assert rep["slowest_rank"] == slow and rep["stragglers"] == [slow], rep
    assert 2.5 <= rep["slowest_vs_median"] <= 3.5, rep
    assert [e["device_key"] for e in rep["per_rank"]] == [100, 101, 102]
    assert rep["per_rank"][slow]["wall_ms"] > 2.5 * rep["per_rank"][0]["wall_ms"]


def test_launch_reports_signal_exit_as_128_plus_signal(tmp_path):
    """dist.launch: a rank killed by a signal (returncode -k) reports 128 + k."""
    D = _load_dist()
    script = tmp_path / "die.py"
    script.write_text("import os, signal\nif os.environ['RANK'] == '1':\n    os.kill(os.getpid(), signal.SIGKILL)\n"
                      "import time\ntime.sleep(30)\n")
    assert D.launch(2, [str(script)], timeout=60) == 128 + 9

"""Multi-GPU helpers: one process per GPU, streams sharded across ranks.

The round trip has no exchange step (streams are independent), so
the only collectives are the start/stop barrier and the max-over-ranks timing
reduction -- control plane, never data.  Backend "nccl" (= RCCL on ROCm) when
every rank owns its own GPU; "gloo" for CPU tests and for several ranks that
share one device (RCCL rejects two ranks on one GPU).

launch(n, argv) starts n ranks of a script as fresh child processes (the
torch.distributed.run environment contract: RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT), so `bench.py --gpus N` works without an
external launcher.  The parent never touches the GPU.
"""
from __future__ import annotations

import datetime
import os
import signal
import socket
import subprocess
import sys
import time

_backend = None


def env_rank_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def device_for(local_rank: int, n_devices: int) -> int:
    """Device ordinal of a local rank: one rank per GPU, round-robin when there
    are more ranks than GPUs (rehearsal of the N-rank path on a 1-GPU box)."""
    return local_rank % max(1, n_devices)


def init_kwargs(backend: str, device=None) -> dict:
    """init_process_group keywords: RCCL binds the rank's device eagerly
    (device_id), gloo takes none."""
    if backend not in ("nccl", "gloo"):
        raise ValueError(f"backend must be 'nccl' (RCCL) or 'gloo', got {backend!r}")
    return {"device_id": device} if (backend == "nccl" and device is not None) else {}


INIT_TIMEOUT_S = 120.0


def init(backend: str, device=None, timeout_s: float = INIT_TIMEOUT_S):
    """Join the process group.  `timeout_s` bounds the rendezvous and every
    collective: a rank that never arrives fails the others in bounded time
    instead of leaving them blocked in RCCL."""
    global _backend
    import torch.distributed as dist
    rank, world, _ = env_rank_world()
    kw = init_kwargs(backend, device)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _backend = backend
    return rank, world


def device_key(device=None) -> int:
    """An id of the physical device a rank runs on (PCI domain / bus / device
    when torch reports them, else the ordinal), so ranks can count distinct GPUs."""
    if device is None:
        return -1
    import torch
    try:
        p = torch.cuda.get_device_properties(device)
        dom, bus, dv = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if bus is not None:
            return (int(dom or 0) << 16) | (int(bus) << 8) | int(dv or 0)
    except Exception:  # noqa: BLE001 -- an id is a report, never fatal
        pass
    return int(getattr(device, "index", device) or 0)


def observed_world(device=None) -> dict:
    """What the process group really holds, seen from every rank: the backend,
    the world size the group reports and the distinct devices its ranks run on
    (an all-gather of device_key over the group)."""
    import torch
    import torch.distributed as dist
    key = device_key(device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return {"backend": _backend or "none", "world": 1, "devices": 1 if key >= 0 else 0, "device_keys": [key]}
    world = dist.get_world_size()
    t = torch.tensor([key], dtype=torch.int64, device=reduce_device(device))
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    keys = [int(v.item()) for v in out]
    return {"backend": dist.get_backend(), "world": world, "devices": len(set(keys)), "device_keys": keys}


def stream_range(total_streams: int, world: int, rank: int):
    """Contiguous block of streams for `rank` ([g*S/G, (g+1)*S/G))."""
    lo = total_streams * rank // world
    hi = total_streams * (rank + 1) // world
    return lo, hi


def barrier():
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def reduce_device(device=None):
    """Where the timing reduction's tensor lives: on the rank's GPU under RCCL
    (which reduces device memory only), on the host under gloo."""
    return device if (_backend == "nccl" and device is not None) else "cpu"


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=reduce_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(values, device=None) -> list:
    """Every rank's list of floats, in rank order (an all-gather; one rank: [values])."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in values]
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [vals]
    t = torch.tensor(vals, dtype=torch.float64, device=reduce_device(device))
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(x) for x in o.cpu().tolist()] for o in out]


STRAGGLER_RATIO = 1.25  # a rank this much slower than the median is named


def rank_report(kernel_ms, wall_ms, device_keys) -> dict:
    """Per-rank timings of a weak-scaling phase and who set the max: each rank's
    device key, mean kernel time and wall time; the slowest rank by wall time, its
    ratio to the median, and `stragglers` (ranks >= STRAGGLER_RATIO x the median
    wall time, worst first) -- so a first multi-GPU run says which GPU held it back."""
    n = len(wall_ms)
    order = sorted(range(n), key=lambda r: wall_ms[r])
    med = wall_ms[order[n // 2]] if n % 2 else 0.5 * (wall_ms[order[n // 2 - 1]] + wall_ms[order[n // 2]])
    slow = order[-1]
    ratio = (wall_ms[slow] / med) if med > 0 else 1.0
    strag = sorted((r for r in range(n) if med > 0 and wall_ms[r] >= STRAGGLER_RATIO * med),
                   key=lambda r: -wall_ms[r])
    return {
        "per_rank": [{"rank": r, "device_key": int(device_keys[r]) if r < len(device_keys) else None,
                      "kernel_ms": round(float(kernel_ms[r]), 4), "wall_ms": round(float(wall_ms[r]), 4)}
                     for r in range(n)],
        "slowest_rank": slow,
        "slowest_vs_median": round(ratio, 3),
        "stragglers": strag,
    }


def finalize():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _stop(procs, grace: float = 5.0):
    """SIGTERM every live child, SIGKILL what is still alive after `grace` s."""
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t_end = time.monotonic() + grace
    for p in procs:
        while p.poll() is None and time.monotonic() < t_end:
            time.sleep(0.05)
        if p.poll() is None:
            p.kill()
            p.wait()


def launch(n: int, argv: list[str], timeout: float | None = None, poll_s: float = 0.1) -> int:
    """Run `python argv...` as n ranks on this node; returns 0 when every rank
    succeeded, else the exit code of the first failure seen (ranks exiting in the
    same poll interval: the lowest rank; a rank killed by signal k: 128 + k).

    All children are polled together: the first non-zero exit stops the other
    ranks at once (they would otherwise wait in a collective for the dead rank),
    and `timeout` (seconds, None: no limit) stops the whole job with 124.
    Children are fresh processes started before anything in this process has
    touched the GPU (no exec from a GPU-initialised process)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    t0 = time.monotonic()
    try:
        for r in range(n):
            e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable] + argv, env=e))
        while True:
            codes = [p.poll() for p in procs]
            # the first failure seen (in rank order within one poll); a rank killed by
            # signal k (returncode -k) reports 128 + k, as a shell does
            bad = [c if c > 0 else 128 - c for c in codes if c not in (None, 0)]
            if bad:
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            if timeout is not None and time.monotonic() - t0 > timeout:
                return 124
            time.sleep(poll_s)
    finally:
        _stop(procs)

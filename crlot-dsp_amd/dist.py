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

import os
import socket
import subprocess
import sys

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


def init(backend: str, device=None):
    global _backend
    import torch.distributed as dist
    rank, world, _ = env_rank_world()
    kw = init_kwargs(backend, device)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, **kw)
    _backend = backend
    return rank, world


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


def launch(n: int, argv: list[str], timeout: float | None = None) -> int:
    """Run `python argv...` as n ranks on this node; returns the worst exit code.

    Children are fresh processes started before anything in this process has
    touched the GPU (no exec from a GPU-initialised process)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
               WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable] + argv, env=e))
    rc = 0
    try:
        for p in procs:
            code = p.wait(timeout=timeout)
            if code != 0 and rc == 0:
                rc = code
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc

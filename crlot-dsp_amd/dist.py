"""Multi-GPU helpers: one process per GPU, streams sharded across ranks.

The round trip has no exchange step (streams are independent), so
the only collectives are the start/stop barrier and the max-over-ranks timing
reduction.  Backend "nccl" (= RCCL on ROCm) on GPUs, "gloo" for CPU tests.
"""
from __future__ import annotations

import os


def env_rank_world():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device=None):
    import torch.distributed as dist
    rank, world, _ = env_rank_world()
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        dist.init_process_group(backend, **kw)
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


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def finalize():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()

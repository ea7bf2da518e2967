"""Batch sharding over the GPUs of one node -- replicas only.

The DA-V2 forward has no exchange step: every image is
independent, so N GPUs run N independent engine replicas on disjoint batch
shards, one process per GPU, no collective on the data path.  This module
holds the host-side bookkeeping: which images a rank owns, the bracketed
timing (barrier + device sync on both sides, max over ranks) and the host
gather of results.  torch.distributed (gloo) is used only for the barrier,
the max-time reduction and the optional result gather -- never RCCL.
"""

from __future__ import annotations

import time
from typing import Callable, List, Optional, Tuple


def shard(global_batch: int, world: int, rank: int) -> Tuple[int, int]:
    """(start, count) of the images rank owns: contiguous, sizes differ by <= 1."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} of {world}")
    if global_batch < 0:
        raise ValueError("negative batch")
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def timed_region(fn: Callable[[], None], steps: int, sync: Callable[[], None],
                 barrier: Optional[Callable[[], None]] = None) -> float:
    """Seconds for `steps` calls of fn, bracketed by barrier + sync on both sides."""
    if barrier:
        barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    t1 = time.perf_counter()
    if barrier:
        barrier()
    return t1 - t0


def max_over_ranks(seconds: float) -> float:
    """Max of a per-rank duration over the process group (identity if none)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_to_rank0(arr) -> Optional[List]:
    """Host gather of each rank's result (numpy) to rank 0, in rank order."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [arr]
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(arr, out, dst=0)
    return out

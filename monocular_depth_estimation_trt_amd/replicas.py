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

import os
import socket
import subprocess
import sys
import time
from typing import Callable, List, Optional, Sequence, Tuple


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


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_local(nprocs: int, script: str, argv: Sequence[str], timeout: Optional[float] = None,
                env: Optional[dict] = None) -> int:
    """Run `python script argv...` as nprocs rank processes of one node (the
    torch.distributed.run environment: RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for them.
    The caller must not have initialised the GPU: the children pick their own
    device from LOCAL_RANK.  stdout/stderr are inherited (rank 0 prints the
    result).  If one rank fails the others are terminated; returns the first
    non-zero exit code, else 0."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = free_port()
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=e))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        if deadline is not None and time.monotonic() > deadline and live:
            for q in live:
                q.kill()
            rc = rc or 124
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc

"""Multi-GPU path = independent replicas on batch shards.  Here
world_size 2 over gloo on the CPU: each rank runs the oracle forward on its
shard, the host gather in rank order must equal the single-process batch,
and the bracketed timing reduces with max over ranks."""

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from monocular_depth_estimation_trt_amd import replicas


def test_shard_partition():
    for n in (0, 1, 7, 8, 33):
        for w in (1, 2, 3, 8):
            parts = [replicas.shard(n, w, r) for r in range(w)]
            assert sum(c for _, c in parts) == n
            starts = [s for s, _ in parts]
            assert starts == sorted(starts) and all(s + c == (parts[i + 1][0] if i + 1 < w else n)
                                                    for i, (s, c) in enumerate(parts))
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1
    with pytest.raises(ValueError):
        replicas.shard(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from monocular_depth_estimation_trt_amd import weights
    from oracle import dav2_ref
    cfg = weights.model_config("vits")
    w = dav2_ref.to_torch(weights.synthetic_state_dict(cfg, 5))
    x = weights.synthetic_images(3, 42, 42, first_seed=20)
    s, c = replicas.shard(3, world, rank)
    out = {}

    def step():
        out["y"] = dav2_ref.forward(w, cfg, x[s:s + c]).numpy()

    el = replicas.timed_region(step, 1, lambda: None, dist.barrier)
    mx = replicas.max_over_ranks(el)
    parts = replicas.gather_to_rank0(out["y"])
    if rank == 0:
        q.put((np.concatenate(parts, 0), mx, el))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_replicas_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, mx, el0 = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from monocular_depth_estimation_trt_amd import weights
    from oracle import dav2_ref
    cfg = weights.model_config("vits")
    ref = dav2_ref.forward(dav2_ref.to_torch(weights.synthetic_state_dict(cfg, 5)), cfg,
                           weights.synthetic_images(3, 42, 42, first_seed=20)).numpy()
    assert got.shape == (3, 42, 42)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    assert mx >= el0 > 0

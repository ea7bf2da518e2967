"""bench.py's multi-GPU launch path on the CPU (replicas only).

`python bench.py --gpus N` without a torch.distributed.run environment spawns
N rank processes itself (replicas.spawn_local) before touching the GPU.  Here
the launcher runs a world-size-2 gloo job whose ranks do exactly the bench's
host-side choreography -- shard, barrier-bracketed timing, per-rank gather,
max over ranks -- and rank 0 writes the line; and bench.main() is checked to
hand off to the launcher with its own argv."""

import json
import os
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from monocular_depth_estimation_trt_amd import replicas  # noqa: E402

RANK_SCRIPT = textwrap.dedent('''
    import json, os, sys, time
    sys.path.insert(0, {root!r})
    import torch.distributed as dist
    from monocular_depth_estimation_trt_amd import replicas
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = int(sys.argv[2])
    first, count = replicas.shard(G, world, rank)
    el = replicas.timed_region(lambda: time.sleep(0.01 * (rank + 1)), 3, lambda: None, dist.barrier)
    per = replicas.gather_to_rank0([first, count, el])
    mx = replicas.max_over_ranks(el)
    if rank == 0:
        with open(sys.argv[1], "w") as f:
            json.dump({{"world": world, "per_rank": per, "max": mx, "value": G * 3 / mx}}, f)
    dist.barrier()
    dist.destroy_process_group()
''')


def test_spawn_local_two_gloo_ranks(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT.format(root=ROOT))
    out = tmp_path / "line.json"
    rc = replicas.spawn_local(2, str(script), [str(out), "3"], timeout=120)
    assert rc == 0
    d = json.loads(out.read_text())
    assert d["world"] == 2
    (f0, c0, e0), (f1, c1, e1) = d["per_rank"]
    assert (f0, c0, f1, c1) == (0, 2, 2, 1)          # 3 items over 2 ranks, contiguous
    assert d["max"] == max(e0, e1) and e1 >= 0.03    # rank 1 sleeps 3 x 20 ms
    assert d["value"] == pytest.approx(9 / d["max"])


def test_spawn_local_propagates_failure(tmp_path):
    script = tmp_path / "bad.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert replicas.spawn_local(2, str(script), [], timeout=60) == 3


def test_bench_self_launches(monkeypatch):
    import bench
    seen = {}

    def fake_spawn(n, script, argv, **kw):
        seen.update(n=n, script=script, argv=list(argv))
        return 0

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(replicas, "spawn_local", fake_spawn)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--encoder", "vitl", "--global-batch", "8"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert seen == {"n": 2, "script": os.path.abspath(bench.__file__),
                    "argv": ["--gpus", "2", "--encoder", "vitl", "--global-batch", "8"]}


def test_bench_rank_work():
    import bench
    a = bench.parse(["--encoder", "vitl", "--global-batch", "8"])
    got = [bench.rank_work(a, 8, r)[:4] for r in range(8)]
    assert got == [(1, r, 8, "strong") for r in range(8)]         # config 3: one image per GPU
    a = bench.parse(["--global-batch", "3"])
    assert [bench.rank_work(a, 4, r)[:2] for r in range(4)] == [(1, 0), (1, 1), (1, 2), (0, 3)]
    a = bench.parse([])
    assert bench.rank_work(a, 4, 2)[:4] == (48, 96, 192, "weak")  # default 48 per GPU

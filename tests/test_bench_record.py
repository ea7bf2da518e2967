"""monocular_depth_estimation_trt_amd.bench keeps the reference's core/bench
semantics (restating the checks of the reference's tests/test_bench.py:30-245
against hand-computed values)."""

import json
import os
import tempfile

import numpy as np
import pytest

from monocular_depth_estimation_trt_amd.bench import (SCHEMA, Bench, load, load_all, measure, measure_staged, record,
                                                      save, summarize_outputs)


def test_stats_arithmetic():
    b = Bench(model="demo", samples_ms=[10.0, 20.0, 30.0, 40.0])
    assert b.iterations == 4 and b.mean_ms == 25.0 and b.fps == 40.0
    s = b.stats()
    assert s["min_ms"] == 10.0 and s["max_ms"] == 40.0


def test_nearest_rank_percentiles():
    b = Bench(model="demo", samples_ms=[float(x) for x in range(1, 101)])
    assert b.pct(50) == 50.0 and b.pct(99) == 99.0 and b.pct(100) == 100.0 and b.pct(0) == 1.0
    for q in (50, 90, 99):
        assert b.pct(q) in b.samples_ms
    one = Bench(model="demo", samples_ms=[7.0])
    assert one.pct(90) == 7.0 and one.stats()["stdev_ms"] == 0.0


def test_empty():
    b = Bench(model="demo")
    assert b.stats() == {} and b.fps == 0.0 and "no samples" in b.report()


def test_measure_warmup_and_sync_inside_timing():
    calls = []
    out, samples = measure(lambda: calls.append(1) or "r", warmup=3, iterations=5, sync=lambda: None)
    assert len(samples) == 5 and len(calls) == 8 and out == "r"
    order = []
    measure(lambda: order.append("run"), warmup=0, iterations=2, sync=lambda: order.append("sync"))
    assert order == ["sync", "run", "sync", "run", "sync"]


def test_measure_staged_probe_per_iteration():
    out, samples, stages = measure_staged(lambda: 1, lambda: {"h2d_ms": 0.5, "compute_ms": 2.0}, warmup=2,
                                          iterations=4, sync=lambda: None)
    assert len(samples) == 4 and stages["h2d_ms"] == [0.5] * 4 and stages["compute_ms"] == [2.0] * 4


def test_summarize_outputs_nonfinite():
    s = summarize_outputs({"depth": np.array([[1.0, 2.0], [np.inf, np.nan]], np.float32)})["depth"]
    assert s["finite"] == 2 and s["nonfinite"] == 2 and s["max"] == 2.0 and abs(s["mean"] - 1.5) < 1e-6
    s = summarize_outputs({"d": np.array([np.inf, np.nan])})["d"]
    assert s["min"] is None and s["mean"] is None


def test_stage_split_and_overhead_clamp():
    b = Bench(model="m", samples_ms=[10.0, 10.0],
              stage_samples_ms={"h2d_ms": [1.0, 1.0], "compute_ms": [4.0, 4.0], "d2h_ms": [1.0, 1.0]})
    s = b.stats()
    assert s["h2d_ms"] == 1.0 and s["compute_ms"] == 4.0 and s["host_overhead_ms"] == 4.0
    assert "compute" in b.report()
    assert "h2d_ms" not in Bench(model="m", samples_ms=[1.0]).stats()
    c = Bench(model="m", samples_ms=[5.0], stage_samples_ms={"h2d_ms": [1.0], "compute_ms": [4.5], "d2h_ms": [1.0]})
    assert c.stats()["host_overhead_ms"] == 0.0


def test_save_load_roundtrip_and_filename():
    b = Bench(model="depth_anything_v2", samples_ms=[5.0, 6.0, 7.0], precision="fp16", profile="bench",
              input_h=518, input_w=518, device="MI355X", warmup=10)
    with tempfile.TemporaryDirectory() as td:
        p = save(b, td)
        assert os.path.basename(p) == "depth_anything_v2_518x518_bench_single_fp16.json"
        d = load(p)
        assert d["schema"] == SCHEMA and d["stats"]["mean_ms"] == 6.0 and d["samples_ms"] == [5.0, 6.0, 7.0]
        assert d["timestamp"] and len(load_all(td)) == 1
        for prec in ("fp32",):
            save(Bench(model="depth_anything_v2", samples_ms=[1.0], precision=prec, input_h=518, input_w=518,
                       device="x"), td)
        assert len(load_all(td)) == 2


def test_schema_mismatch_raises():
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "bad.json")
        json.dump({"schema": SCHEMA + 99}, open(p, "w"))
        with pytest.raises(ValueError):
            load(p)


def test_record_writes_and_reports(capsys):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "bench")
        b = record("depth_anything_v2", [4.0, 5.0], outputs={"depth": np.ones((2, 2), np.float32)},
                   model_input=np.zeros((1, 3, 14, 14), np.float32), out_dir=out, warmup=1, input_h=14,
                   input_w=14, device="test")
        assert b.outputs["depth"]["mean"] == 1.0
        assert os.path.exists(os.path.join(td, "inputs", "depth_anything_v2.npy"))
        assert "[MDET] Average FPS" in capsys.readouterr().out

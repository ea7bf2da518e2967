"""The reference's call sequence (models/depth_anything_v2/onnx2trt.py:93-127,
core/common_runtime.py, core/bench.py) run unchanged against this package:
get_engine -> create_execution_context -> allocate_buffers -> do_inference
(+ StageTimer, IProfiler) -> bench.measure -> bench.record, checked against
the oracle."""

import os
import tempfile

import numpy as np
import pytest

from gpu_util import depth_metrics
from monocular_depth_estimation_trt_amd import bench, common, weights
from monocular_depth_estimation_trt_amd.common_runtime import (StageTimer, allocate_buffers, do_inference,
                                                               free_buffers)

pytestmark = pytest.mark.gpu


def oracle(x, seed=1234):
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    return dav2_ref.forward(dav2_ref.to_torch(weights.synthetic_state_dict(cfg, seed)), cfg, x).numpy()


def test_reference_call_sequence(gpu):
    x = weights.synthetic_images(1, 98, 98, first_seed=4)
    with tempfile.TemporaryDirectory() as td:
        eng_path = os.path.join(td, "engine", "dav2_vits_98_fp16.mdeng")
        output_shape = (1, 98, 98)
        with common.get_engine("synthetic:vits:metric:1234", eng_path, "fp16", None, input_hw=(98, 98)) as engine, \
                engine.create_execution_context() as context:
            assert engine.num_io_tensors == 2
            assert [engine.get_tensor_name(i) for i in range(2)] == ["input", "output"]
            assert engine.get_tensor_shape("input") == (1, 3, 98, 98)
            inputs, outputs, bindings, stream = allocate_buffers(engine, output_shape, profile_idx=0)
            inputs[0].host = x
            outs, samples = bench.measure(
                lambda: do_inference(context, engine=engine, bindings=bindings, inputs=inputs, outputs=outputs,
                                     stream=stream), warmup=2, iterations=5)
            depth = outs[0].reshape(output_shape).copy()
            timer = StageTimer()
            do_inference(context, engine, bindings, inputs, outputs, stream, timer=timer)
            assert set(timer.last) == {"h2d_ms", "compute_ms", "d2h_ms"} and timer.last["compute_ms"] > 0
            timer.free()

            class Prof:
                def __init__(self):
                    self.names = []

                def report_layer_time(self, name, ms):
                    self.names.append(name)

            context.profiler = Prof()
            do_inference(context, engine, bindings, inputs, outputs, stream)
            names = context.profiler.names
            context.profiler = None
            assert "block0.attn" in names and "head.output_conv2" in names and len(names) > 90
            free_buffers(inputs, outputs, stream)
            b = bench.record("depth_anything_v2", samples, outputs={"depth": depth}, out_dir=os.path.join(td, "b"),
                             warmup=2, precision="fp16", input_h=98, input_w=98, engine_path=eng_path, echo=False)
            assert b.engine_bytes > 0 and b.outputs["depth"]["nonfinite"] == 0
        # second get_engine: loaded from the packed file, not rebuilt
        with common.get_engine("synthetic:vits:metric:1234", eng_path, "fp16", None, input_hw=(98, 98)) as e2:
            assert e2.path == eng_path
    m = depth_metrics(depth, oracle(x))
    assert m["rel_mean"] < 5e-3 and m["corr"] > 0.9995, m


def test_dynamic_batch_engine(gpu):
    x = weights.synthetic_images(3, 70, 70, first_seed=9)
    with common.get_engine("synthetic:vits", "", "fp16",
                           dynamic_input_shapes=[[1, 3, 70, 70], [2, 3, 70, 70], [4, 3, 70, 70]]) as engine, \
            engine.create_execution_context() as ctx:
        assert engine.get_tensor_shape("input") == (-1, 3, 70, 70)
        assert engine.get_tensor_profile_shape("input", 0)[-1] == (4, 3, 70, 70)
        inputs, outputs, bindings, stream = allocate_buffers(engine, None, profile_idx=0)
        ctx.set_input_shape("input", (3, 3, 70, 70))
        assert ctx.get_tensor_shape("output") == (3, 70, 70)
        inputs[0].host = x
        # host views are freed with the buffers (as in the reference): copy first
        out = do_inference(ctx, engine, bindings, inputs, outputs, stream)[0][:3 * 70 * 70].reshape(3, 70, 70).copy()
        with pytest.raises(Exception):
            ctx.set_input_shape("input", (5, 3, 70, 70))
        free_buffers(inputs, outputs, stream)
    m = depth_metrics(out, oracle(x))
    assert m["rel_mean"] < 5e-3 and m["corr"] > 0.9995, m


def test_driver_script(gpu):
    from monocular_depth_estimation_trt_amd.models.depth_anything_v2 import run
    with tempfile.TemporaryDirectory() as td:
        d = run.main(["--engine", os.path.join(td, "e.mdeng"), "--iterations", "3", "--warmup", "1",
                      "--src-hw", "300", "400", "--out-dir", os.path.join(td, "bench")])
        assert d.shape == (300, 400) and np.isfinite(d).all() and d.min() >= 1e-3
        assert os.path.exists(os.path.join(td, "bench", "depth_anything_v2_518x518_bench_single_fp16.json"))


@pytest.mark.parametrize("model", ["depth_anything_ac", "distill_any_depth"])
def test_family_drivers(gpu, model):
    """The DA-V2 family drivers (relative head) run the reference sequence;
    distill_any_depth keeps the 518x518 map, depth_anything_ac resizes+clamps."""
    import importlib
    run = importlib.import_module(f"monocular_depth_estimation_trt_amd.models.{model}.run")
    with tempfile.TemporaryDirectory() as td:
        d = run.main(["--engine", os.path.join(td, "e_fp16.mdeng"), "--iterations", "2", "--warmup", "1",
                      "--src-hw", "300", "400", "--out-dir", os.path.join(td, "bench")])
        assert os.path.exists(os.path.join(td, "bench", f"{model}_518x518_bench_single_fp16.json"))
    assert np.isfinite(d).all() and d.min() >= 0.0
    assert d.shape == ((518, 518) if model == "distill_any_depth" else (300, 400))

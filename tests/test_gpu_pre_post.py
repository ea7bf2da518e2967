"""uint8 NHWC input and on-device post-process, through
the C ABI, against oracle/pre_post.py (the reference's uint8 preamble,
core/onnx_tools.py:87-219, and post-process, onnx2trt.py:111-117).

Parity bars:
* the preamble computes the reference's fp32 ops in the same order, so the
  patch operand is bit-identical to the f16 rounding of the host-normalised
  image, and the uint8 engine's depth map is bit-identical to the float
  engine's on that host-normalised image (same kernels downstream);
* the post-process is fp32 bilinear (align_corners) + clamp: |d - ref| <=
  1e-5 * max(1, |ref|) (fp32 rounding of the 4-tap blend, no fp16 involved).
"""

import os
import tempfile

import numpy as np
import pytest
import torch

from gpu_util import op, ptr, stream

from monocular_depth_estimation_trt_amd import common, pack, weights
from monocular_depth_estimation_trt_amd.common_runtime import allocate_buffers, do_inference, free_buffers
from monocular_depth_estimation_trt_amd.engine import DataType, Engine
from oracle import pre_post

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hw", [(28, 42), (98, 98), (518, 518)])
def test_patch_prep_u8_bit_exact(gpu, hw):
    h, w = hw
    u = weights.synthetic_images_u8(2, h, w, first_seed=11)
    ref = pre_post.patch_matrix(pre_post.uint8_preamble(u))
    mean = torch.tensor(pre_post.MEAN, dtype=torch.float32, device="cuda")
    std = torch.tensor(pre_post.STD, dtype=torch.float32, device="cuda")
    du = torch.from_numpy(u).cuda()
    P = torch.full(ref.shape, float("nan"), dtype=torch.float16, device="cuda")
    op("mde_op_patch_prep_u8", ptr(du), 2, h, w, 255.0, ptr(mean), ptr(std), ptr(P), stream())
    got = P.cpu().numpy()
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))


def _run(eng, x):
    ctx = eng.create_execution_context()
    B = x.shape[0]
    xin = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    H, W = eng.input_hw
    out = torch.empty(B, H, W, device="cuda")
    ctx.set_input_shape(eng.input_name, x.shape)
    ctx.set_tensor_address(eng.input_name, xin.data_ptr())
    ctx.set_tensor_address("output", out.data_ptr())
    ctx.execute_async_v3(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    ctx.destroy()
    return y


def test_uint8_engine_equals_float_engine(gpu):
    h = w = 98
    u = weights.synthetic_images_u8(2, h, w, first_seed=5)
    blob_f, _ = pack.synthetic_blob("vits", "metric", h, w)
    blob_u, _ = pack.synthetic_blob("vits", "metric", h, w, input_format="uint8_nhwc")
    prof_f = ((1, 3, h, w), (2, 3, h, w), (2, 3, h, w))
    prof_u = ((1, h, w, 3), (2, h, w, 3), (2, h, w, 3))
    with Engine.from_bytes(blob_u, 0, profile=prof_u) as eu, Engine.from_bytes(blob_f, 0, profile=prof_f) as ef:
        assert eu.input_name == "image_u8" and eu.input_format == "uint8_nhwc"
        assert eu.get_tensor_dtype("image_u8") == DataType.UINT8
        assert eu.get_tensor_shape("image_u8") == (-1, h, w, 3)
        yu = _run(eu, u)
        yf = _run(ef, pre_post.uint8_preamble(u))
    assert np.isfinite(yu).all()
    assert np.array_equal(yu, yf)


def test_uint8_dropin_call_sequence(gpu):
    """get_engine(input_format='uint8_nhwc') + allocate_buffers/do_inference
    with a uint8 host array (0.8 MB H2D at 518 instead of 3.2 MB)."""
    h = w = 70
    u = weights.synthetic_images_u8(1, h, w, first_seed=2)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "dav2_vits_70_u8_fp16.mdeng")
        with common.get_engine("synthetic:vits", path, "fp16", None, input_hw=(h, w),
                               input_format="uint8_nhwc") as engine, \
                engine.create_execution_context() as ctx:
            inputs, outputs, bindings, st = allocate_buffers(engine, (1, h, w), profile_idx=0)
            assert inputs[0].host.dtype == np.uint8 and inputs[0].nbytes == h * w * 3
            inputs[0].host = u
            y = do_inference(ctx, engine, bindings, inputs, outputs, st)[0].reshape(1, h, w).copy()
            free_buffers(inputs, outputs, st)
        with pytest.raises(ValueError):
            common.get_engine("synthetic:vits", "", "fp16", None, input_format="uint8_nchw")
    with Engine.from_bytes(pack.synthetic_blob("vits", "metric", h, w)[0], 0) as ef:
        yf = _run(ef, pre_post.uint8_preamble(u))
    assert np.array_equal(y, yf)


@pytest.mark.parametrize("src", [(518, 518, 2268, 3024), (518, 518, 300, 400), (37, 53, 518, 518), (5, 7, 1, 9)])
def test_depth_postprocess(gpu, src):
    ih, iw, oh, ow = src
    g = torch.Generator().manual_seed(ih * 1000 + oh)
    d = (torch.rand(2, ih, iw, generator=g) * 30.0 - 2.0).numpy()  # crosses both clamp bounds
    d[0, 0, 0] = 5e3
    ref = pre_post.postprocess(d, oh, ow)
    din = torch.from_numpy(d).cuda()
    out = torch.full((2, oh, ow), float("nan"), device="cuda")
    op("mde_op_depth_postprocess", ptr(din), 2, ih, iw, ptr(out), oh, ow, 1e-3, 1e3, stream())
    got = out.cpu().numpy()
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    assert np.isfinite(got).all() and err.max() <= 1e-5, err.max()
    assert got.min() >= 1e-3 and got.max() <= 1e3


def test_driver_uint8_and_device_postprocess(gpu):
    from monocular_depth_estimation_trt_amd.models.depth_anything_v2 import run
    with tempfile.TemporaryDirectory() as td:
        args = ["--engine", os.path.join(td, "e_fp16.mdeng"), "--iterations", "2", "--warmup", "1",
                "--src-hw", "300", "400", "--out-dir", os.path.join(td, "bench")]
        d_dev = run.main(args + ["--input-format", "uint8_nhwc"])
        d_host = run.main(args + ["--input-format", "uint8_nhwc", "--host-postprocess"])
        assert os.path.exists(os.path.join(td, "e_u8_fp16.mdeng"))
        assert os.path.exists(os.path.join(td, "bench", "depth_anything_v2_518x518_bench_u8_fp16.json"))
    assert d_dev.shape == (300, 400) and d_dev.min() >= 1e-3
    assert np.abs(d_dev - d_host).max() <= 1e-5 * max(1.0, float(np.abs(d_host).max()))

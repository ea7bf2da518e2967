"""The fused ViT-S MLP kernel (csrc/mlp_fused.hip: fc1 + GELU + fc2 +
LayerScale residual in one launch) through the C ABI: against a torch fp32
reference of the same op (the hidden activation rounded to f16, as the
unfused engine stores it), with row tails; and the DA-V2 engine with the
fused MLP forced on against the same engine with it off.

Tolerance: |x_out - ref| <= 2 % of the largest residual update + 1e-3
(f16 operands, fp32 accumulation; GELU's fitted form may flip the f16
rounding of single hidden values); engine fused vs unfused within 0.1 % of
the depth range."""

import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_util import op, pad_w, ptr, stream

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [100, 1370, 33000])
def test_mlp_residual_op(gpu, M):
    torch.manual_seed(M)
    D, Hd = 384, 1536
    a = torch.randn(M, D).half()
    w1, b1 = torch.randn(Hd, D) / D ** 0.5, 0.02 * torch.randn(Hd)
    w2, b2 = torch.randn(D, Hd) / Hd ** 0.5, 0.02 * torch.randn(D)
    ls = 0.5 + 0.05 * torch.randn(D)
    x = torch.randn(M, D)
    h = F.gelu(a.float() @ w1.half().float().T + b1).half().float()
    upd = ls * (h @ w2.half().float().T + b2)
    ref = x + upd
    xd = x.cuda()
    op("mde_op_mlp_residual", ptr(a.cuda()), M, ptr(pad_w(w1.cuda())), D, ptr(b1.cuda()), ptr(pad_w(w2.cuda())), Hd,
       ptr(b2.cuda()), ptr(ls.cuda()), ptr(xd), D, Hd, stream())
    err = (xd.cpu() - ref).abs()
    assert float(err.max()) <= 2e-2 * float(upd.abs().max()) + 1e-3, float(err.max())


def test_mlp_residual_op_rejects_other_widths(gpu):
    from monocular_depth_estimation_trt_amd._lib import MDEError
    z = torch.zeros(64, 768, dtype=torch.float16, device="cuda")
    with pytest.raises(MDEError):
        op("mde_op_mlp_residual", ptr(z), 64, ptr(z), 768, ptr(z), ptr(z), 3072, ptr(z), ptr(z), ptr(z), 768, 3072,
           stream())


def _run(blob, x):
    from monocular_depth_estimation_trt_amd.engine import Engine
    B = x.shape[0]
    eng = Engine.from_bytes(blob, 0, profile=((1,) + x.shape[1:], x.shape, x.shape))
    ctx = eng.create_execution_context()
    xin = torch.from_numpy(x).cuda()
    out = torch.empty(B, x.shape[2], x.shape[3], device="cuda")
    ctx.set_input_shape("input", x.shape)
    ctx.set_tensor_address("input", xin.data_ptr())
    ctx.set_tensor_address("output", out.data_ptr())
    ctx.execute_async_v3(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    ctx.destroy()
    eng.destroy()
    return y


def test_engine_fused_mlp_equals_unfused(gpu):
    from monocular_depth_estimation_trt_amd import pack, weights
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    x = weights.synthetic_images(2, 98, 98, first_seed=100)
    blob = pack.pack_bytes(sd, cfg, 98, 98)
    outs = {}
    os.environ["MDE_SPLITK"] = "0"  # compare against the plain (unsplit) fc2
    for mode in ("0", "2"):
        os.environ["MDE_FUSED_MLP"] = mode
        try:
            outs[mode] = _run(blob, x)
        finally:
            os.environ.pop("MDE_FUSED_MLP", None)
    os.environ.pop("MDE_SPLITK", None)
    d = float(np.abs(outs["0"] - outs["2"]).max())
    print("fused vs unfused max_abs", d)
    assert np.isfinite(outs["2"]).all()
    assert d <= 1e-3 * float(np.abs(outs["0"]).max()), d

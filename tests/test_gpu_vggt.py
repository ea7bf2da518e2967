"""VGGT's depth path on the HIP engine, through the C
ABI, against the oracle (oracle/vggt_ref.py; partially pinned, see its
header): the "tiny" preset (98x98, 7x7 patches, D 128) for one and two
frames, "vggt_1b_shallow" -- every kernel shape of VGGT-1B at 518^2
(D 1024, 16 heads, T 1374, the 2048-wide taps, the full DPT decoder) with
2 + 4 blocks -- and the bench model "vggt_1b" itself (24 + 24 blocks, one and
two frames; the oracle takes ~10 s per frame on the box's cores).

Tolerance (fp16 operands, fp32 accumulation vs the fp32 oracle), stated
per case in _check's callers at ~3x the measured error: depth rel_mean <=
2e-3 (tiny) / 3e-3 (VGGT-1B widths), Pearson corr >= 0.99999, per pixel
|d - d_ref| <= 0.012-0.02.  The bandwidth kernels (q/k norm + RoPE, tap
LayerNorm) are held to f16 rounding of the fp32 reference.
"""

import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from gpu_util import depth_metrics, op, ptr, stream

from monocular_depth_estimation_trt_amd import pack_vggt, weights_vggt as WV
from monocular_depth_estimation_trt_amd.engine import Engine
from oracle import vggt_ref

pytestmark = pytest.mark.gpu


def run_engine(blob, x: np.ndarray, graph=True):
    """x [B, S, 3, H, W] -> depth [B, S, H, W, 1] through the engine API."""
    eng = Engine.from_bytes(blob, 0, profile=((1,) + x.shape[1:], x.shape, x.shape))
    assert [eng.get_tensor_name(i) for i in range(eng.num_io_tensors)] == ["images", "depth"]
    assert eng.get_tensor_profile_shape("images", 0)[2] == x.shape
    ctx = eng.create_execution_context()
    ctx.set_graph_mode(graph)
    xin = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    out = torch.full(x.shape[:2] + x.shape[3:] + (1,), float("nan"), device="cuda")
    ctx.set_input_shape("images", x.shape)
    assert ctx.get_tensor_shape("depth") == tuple(out.shape)
    ctx.set_tensor_address("images", xin.data_ptr())
    ctx.set_tensor_address("depth", out.data_ptr())
    ctx.execute_async_v3(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    y = out.cpu().numpy()
    ctx.destroy()
    eng.destroy()
    return y


def _case(preset, batch, frames, seed=2468, img_seed=300):
    cfg = WV.vggt_config(preset)
    sd = WV.synthetic_state_dict(cfg, seed)
    x = WV.synthetic_images(batch, frames, cfg["img"], first_seed=img_seed)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    ref = vggt_ref.forward(vggt_ref.to_torch(sd), cfg, x).numpy()
    return cfg, sd, x, ref, pack_vggt.pack_bytes(sd, cfg, frames)


@pytest.fixture(scope="module")
def tiny_b2(gpu):
    return _case("tiny", 2, 1)


@pytest.fixture(scope="module")
def tiny_s2(gpu):
    return _case("tiny", 1, 2)


# Tolerances: about 3x the error measured on MI355X (profiles/r02_gpu_tests.log:
# tiny B=2 rel 6.6e-4 / max_abs 0.0037, tiny S=2 7.1e-4 / 0.0061, VGGT-1B
# widths at 518^2 9.3e-4 / 0.0055, corr >= 0.999997 everywhere), so a
# numerical regression of a few x fails.  Against the oracle only: the VGGT
# aggregator is parity-unpinned.
def _check(y, ref, what, rel=2e-3, max_abs=0.02, corr=0.99999):
    m = depth_metrics(y, ref)
    print(what, m, "ref range", float(ref.min()), float(ref.max()), flush=True)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    assert np.isfinite(y).all()
    assert m["rel_mean"] <= rel, m
    assert m["corr"] >= corr, m
    assert m["max_abs"] <= max_abs, m


def test_tiny_batch2_matches_oracle(tiny_b2):
    cfg, sd, x, ref, blob = tiny_b2
    _check(run_engine(blob, x), ref, "vggt tiny B=2 S=1", rel=2e-3, max_abs=0.012)


def test_tiny_two_frames_matches_oracle(tiny_s2):
    """S = 2: global attention over both frames, special-token set 1 on frame 1."""
    cfg, sd, x, ref, blob = tiny_s2
    _check(run_engine(blob, x), ref, "vggt tiny B=1 S=2", rel=2e-3, max_abs=0.02)


def test_graph_equals_eager_and_batch_consistency(tiny_b2):
    cfg, sd, x, ref, blob = tiny_b2
    yg = run_engine(blob, x, graph=True)
    ye = run_engine(blob, x, graph=False)
    assert np.array_equal(yg, ye)
    y1 = run_engine(blob, x[1:2])       # item 1 alone == item 1 of the batch
    assert np.array_equal(y1[0], yg[1])


def test_vggt_1b_shallow_518_matches_oracle(gpu):
    cfg, sd, x, ref, blob = _case("vggt_1b_shallow", 1, 1)
    assert ref.shape == (1, 1, 518, 518, 1)
    _check(run_engine(blob, x), ref, "vggt_1b_shallow 518 B=1", rel=3e-3, max_abs=0.017)


@pytest.mark.parametrize("frames", [1, 2])
def test_vggt_1b_full_518_matches_oracle(gpu, frames):
    """The bench model itself (bench.py --model vggt: "vggt_1b" = 24 DINOv2
    blocks + 24 frame/global block pairs, the DPT taps after aggregator
    blocks 4, 11, 17, 23 -- weights_vggt.py), B = 1 at 518^2, one frame and
    two (global attention over 2 x 1374 tokens, special-token set 1 on frame
    1), against the oracle: the tap indexing and the error growth over the
    real depth, which the shallow preset cannot show.  Aggregator parity
    unpinned (oracle/vggt_ref.py header: the reference holds nothing to pin
    it against); the bars are ~3x the error measured on MI355X
    (gpurun_out r4s3: S=1 rel 7.7e-4, max_abs 0.0086, corr 0.9999947; S=2
    7.7e-4 / 0.0088 / 0.9999947; depth range 0.39-4.35)."""
    cfg, sd, x, ref, blob = _case("vggt_1b", 1, frames)
    assert ref.shape == (1, frames, 518, 518, 1)
    _check(run_engine(blob, x), ref, f"vggt_1b (24 + 24 blocks) 518 B=1 S={frames}", rel=2.5e-3, max_abs=0.026,
           corr=0.99998)


def test_engine_rejects_bad_shapes(tiny_b2):
    cfg, sd, x, ref, blob = tiny_b2
    eng = Engine.from_bytes(blob, 0, profile=((1,) + x.shape[1:],) * 3)
    ctx = eng.create_execution_context()
    with pytest.raises(RuntimeError):
        ctx.set_input_shape("images", (1, 2) + x.shape[2:])     # engine packed for S = 1
    with pytest.raises(RuntimeError):
        ctx.set_input_shape("images", x.shape[:1] + x.shape[2:])  # rank 4
    with pytest.raises(RuntimeError):
        ctx.set_tensor_address("output", 0)   # DA-V2's name: not a VGGT binding
    ctx.destroy()
    eng.destroy()


@pytest.mark.parametrize("frames", [1, 2])
def test_qk_norm_rope_op(gpu, frames):
    """q/k LayerNorm(64) + 2D RoPE + q scale on head-major rows, vs the oracle's
    layer_norm + rope2d (frames = 2: the global-attention token order)."""
    torch.manual_seed(frames)
    gh = gw = 7
    npre, H, nseq = 5, 3, 2
    P = npre + gh * gw
    T = frames * P
    Tpad = -(-T // 64) * 64
    BH = nseq * H
    q = torch.zeros(BH, Tpad, 64)
    k = torch.zeros(BH, Tpad, 64)
    q[:, :T] = torch.randn(BH, T, 64) * 1.5 + 0.3
    k[:, :T] = torch.randn(BH, T, 64) * 0.7 - 0.2
    qg, qb, kg, kb = (1 + 0.1 * torch.randn(64), 0.1 * torch.randn(64), 1 + 0.1 * torch.randn(64),
                      0.1 * torch.randn(64))
    cos, sin = pack_vggt.rope_tables(gw + 2)
    qs = 0.125 * 1.4426950408889634
    pos = vggt_ref.rope_positions(gh, gw, npre).repeat(frames, 1)
    qh, kh = q.half(), k.half()
    ref_q = vggt_ref.rope2d(F.layer_norm(qh[:, :T].float(), (64,), qg, qb, 1e-5), pos) * qs
    ref_k = vggt_ref.rope2d(F.layer_norm(kh[:, :T].float(), (64,), kg, kb, 1e-5), pos)
    qd, kd = qh.cuda(), kh.cuda()
    op("mde_op_qk_norm_rope", ptr(qd), ptr(kd), ptr(qg.cuda()), ptr(qb.cuda()), ptr(kg.cuda()), ptr(kb.cuda()), BH, T,
       Tpad, P, npre, gw, ptr(torch.from_numpy(cos).cuda()), ptr(torch.from_numpy(sin).cuda()), qs, 1e-5, stream())
    for got, ref in ((qd, ref_q), (kd, ref_k)):
        g = got.float().cpu()
        err = (g[:, :T] - ref).abs()
        assert float(err.max()) <= 4e-3 * float(ref.abs().max()), float(err.max())
        assert float(g[:, T:].abs().max()) == 0.0          # pad rows untouched


@pytest.mark.parametrize("D", [128, 1024])
def test_tap_concat_ln_op(gpu, D):
    torch.manual_seed(D)
    nseq, npre, npch = 3, 5, 49
    T = npre + npch
    xa = torch.randn(nseq, T, D) * 2 + 0.5
    xb = torch.randn(nseq, T, D) * 0.5 - 1.0
    g = 1 + 0.1 * torch.randn(2 * D)
    b = 0.1 * torch.randn(2 * D)
    ref = F.layer_norm(torch.cat([xa, xb], -1)[:, npre:], (2 * D,), g, b, 1e-5).reshape(nseq * npch, 2 * D)
    out = torch.empty(nseq * npch, 2 * D, dtype=torch.float16, device="cuda")
    op("mde_op_tap_concat_ln", ptr(xa.cuda()), ptr(xb.cuda()), nseq, T, npre, D, ptr(g.cuda()), ptr(b.cuda()), 1e-5,
       ptr(out), stream())
    err = (out.float().cpu() - ref).abs()
    assert float(err.max()) <= 2e-3 * float(ref.abs().max()) + 1e-3, float(err.max())

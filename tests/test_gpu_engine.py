"""End-to-end parity of the HIP engine (through the C ABI) against the oracle
and the committed golden fixtures (HF-pinned, tests/golden/make_golden.py).

Tolerance (north_star: "fp16 depth maps ... within a stated per-pixel
tolerance"): the engine computes with fp16 operands and fp32 accumulation.
Against the fp32 reference (2-3x the error measured on MI355X,
profiles/r02_gpu_tests.log; default "fp16" engines, f16 residual stream:
ViT-S 518 rel 7.1e-4 / 0.035 m, ViT-L 518 rel 3.9e-4 / 0.038 m; "fp32"
engines 6.1e-4 / 0.028 m and 3.1e-4 / 0.029 m):
    ViT-S/B/L:      rel_mean <= 0.15 %,  max |d - d_ref| <= 0.003 * max_depth
    relative heads: rel_mean <= 0.5 %, max_abs <= 0.005 * max |ref| (ReLU
                    output: mean |ref| is small; measured 2.1e-3 / 0.0033)
    all:            Pearson corr >= 0.9999
(0.06 m for the metric head's 20 m).  The 518x518 HF goldens are
stored in f16 (<= 7.9e-3 quantisation), added to the max_abs bound there.
The reference's own TensorRT fp16 engine measured rel_mean 0.170 %, max_abs
0.0239 m, corr 0.99998 against its fp32 ONNX (reports/accuracy.json:32-35).
Shape and index handling must be exact (output [B,H,W], tap indices, NHWC
bookkeeping): a wrong index shows up as corr << 1.
"""

import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from gpu_util import depth_metrics

from monocular_depth_estimation_trt_amd import pack, weights
from monocular_depth_estimation_trt_amd.engine import Engine

pytestmark = pytest.mark.gpu

CORR = 0.9999
TOL = {"vits": (1.5e-3, 0.003), "vitb": (1.5e-3, 0.003), "vitl": (1.5e-3, 0.003),  # (rel_mean, max_abs / max_depth)
       # relative heads end in a ReLU: most of the map sits near 0, so the same
       # absolute error is a larger fraction of mean |ref| (measured 1.9e-3)
       "relative": (5e-3, 0.005)}
F16_Q = 7.9e-3   # f16 storage quantisation of the 518^2 goldens


def run_engine(blob, x: np.ndarray, graph=True, max_batch=None):
    B = x.shape[0]
    eng = Engine.from_bytes(blob, 0, profile=((1, 3) + x.shape[2:], (B, 3) + x.shape[2:],
                                              (max_batch or B, 3) + x.shape[2:]))
    ctx = eng.create_execution_context()
    ctx.set_graph_mode(graph)
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


def check(y, ref, max_depth, what, encoder="vits", extra_abs=0.0):
    rel_bar, abs_frac = TOL[encoder]
    m = depth_metrics(y, ref)
    print(what, m, flush=True)
    assert np.isfinite(y).all(), what
    assert m["rel_mean"] <= rel_bar, (what, m)
    assert m["corr"] >= CORR, (what, m)
    assert m["max_abs"] <= abs_frac * max_depth + extra_abs, (what, m)
    return m


@pytest.mark.parametrize("name", ["dav2_vits_metric_98", "dav2_vits_relative_98", "dav2_vitb_relative_98", "dav2_vitl_metric_98"])
def test_engine_vs_golden_98(gpu, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    enc, dt = str(z["encoder"]), str(z["depth_type"])
    cfg = weights.model_config(enc, dt)
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    assert weights.state_dict_digest(sd) == str(z["weights_sha256"]), "synthetic weight generator drifted"
    size = int(z["size"])
    blob = pack.pack_bytes(sd, cfg, size, size)
    y = run_engine(blob, z["input"])
    ref = z["output_hf"]
    assert y.shape == ref.shape
    md = cfg["max_depth"] if dt == "metric" else max(float(np.abs(ref).max()), 1e-3)
    check(y, ref, md, name, enc if dt == "metric" else "relative")


@pytest.mark.parametrize("name,encoder", [("dav2_vits_metric_518", "vits"), ("dav2_vitl_metric_518", "vitl")])
def test_engine_vs_golden_518(gpu, name, encoder):
    """Full 518x518 map at B=1 against HF.  ViT-L at B=1 is BASELINE config
    3's per-GPU unit: its fc2 runs split-K, 128^2 tiles x 4 slices of the K loop
    (gemm.hip launch_gemm, E_RESID split), reduced in slice order."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    assert weights.state_dict_digest(sd) == str(z["weights_sha256"]), "synthetic weight generator drifted"
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    x = weights.synthetic_images(1, 518, 518, first_seed=int(z["input_first_seed"]))
    y = run_engine(blob, x)
    assert y.shape == (1, 518, 518)
    check(y, z["output_hf_f16"].astype(np.float32), 20.0, f"{name} B=1 vs HF golden (full map)", encoder,
          extra_abs=F16_Q)
    assert abs(float(y.mean()) - float(z["out_mean"])) < 2e-3 * abs(float(z["out_mean"]))
    assert abs(float(y.std()) - float(z["out_std"])) < 5e-3 * float(z["out_std"])


def test_engine_vs_oracle_518_full(gpu):
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    x = weights.synthetic_images(2, 518, 518, first_seed=0)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, 518, 518), x)
    check(y, ref, 20.0, "518 B=2 vs oracle")


def test_engine_518_b8_vs_oracle(gpu):
    """B=8 at 518x518 (the 128^2 GEMM tiles and 8-wave attention of the
    large-batch bench path); every image against the oracle."""
    from oracle import dav2_ref
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 4321)
    x = weights.synthetic_images(8, 518, 518, first_seed=60)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, 518, 518), x)
    check(y, ref, 20.0, "518 B=8 vs oracle")


def test_engine_vitl_518_b2_vs_oracle(gpu):
    """ViT-L 518x518, B=2 (unsplit fc2: 688 64^2 tiles) against the oracle."""
    from oracle import dav2_ref
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = weights.model_config("vitl", "metric")
    sd = weights.synthetic_state_dict(cfg, 77)
    x = weights.synthetic_images(2, 518, 518, first_seed=40)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, 518, 518), x)
    check(y, ref, 20.0, "vitl 518 B=2 vs oracle", "vitl")


def test_engine_nonsquare_vs_oracle(gpu):
    """126x182 (9x13 patches): pos-embed interpolation, odd 4th-scale size."""
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 99)
    x = weights.synthetic_images(2, 126, 182, first_seed=3)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, 126, 182), x)
    assert y.shape == (2, 126, 182)
    check(y, ref, 20.0, "126x182 vs oracle")


def test_batch_and_graph_consistency(gpu):
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 5)
    blob = pack.pack_bytes(sd, cfg, 98, 98)
    x = weights.synthetic_images(3, 98, 98, first_seed=11)
    y3 = run_engine(blob, x, graph=True)
    y3e = run_engine(blob, x, graph=False)
    assert np.array_equal(y3, y3e), "graph replay must equal eager launches bit for bit"
    y3b = run_engine(blob, x, graph=True)
    assert np.array_equal(y3, y3b), "engine must be deterministic"
    for i in range(3):
        yi = run_engine(blob, x[i:i + 1], max_batch=4)
        m = depth_metrics(yi, y3[i:i + 1])
        assert m["max_abs"] < 0.05 and m["rel_mean"] < 1e-3, (i, m)


@pytest.mark.parametrize("encoder,size", [("vits", 98), ("vitl", 518)])
def test_fc2_splitk_matches_unsplit(gpu, encoder, size):
    """Small-batch contexts split fc2's K loop (gemm.hip launch_gemm: ViT-S at
    98^2 4 slices of 64^2 tiles, ViT-L at 518^2 4 slices of 128^2 tiles --
    config 3's B=1); the slices are
    summed in order, so the result is deterministic and equal to the unsplit
    GEMM up to fp32 reassociation."""
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 5)
    blob = pack.pack_bytes(sd, cfg, size, size)
    x = weights.synthetic_images(1, size, size, first_seed=21)
    y_split = run_engine(blob, x, graph=True)
    assert np.array_equal(y_split, run_engine(blob, x, graph=False)), "split-K must be deterministic"
    os.environ["MDE_SPLITK"] = "0"
    try:
        y_plain = run_engine(blob, x)
    finally:
        os.environ.pop("MDE_SPLITK", None)
    m = depth_metrics(y_split, y_plain)
    print(f"split-K vs unsplit {encoder} {size}", m)
    # the fp32 reassociation is amplified by the downstream f16 roundings
    # (measured ViT-S 0.026 m / 6.6e-4, ViT-L 0.036 m / 6.2e-4)
    assert m["max_abs"] < 0.08 and m["rel_mean"] < 1.5e-3, m


@pytest.mark.parametrize("encoder,size,B", [("vits", 98, 2), ("vitl", 518, 1)])
def test_dpt_fork_bit_exact(gpu, encoder, size, B):
    """Small grids run the reassemble + layerN_rn branch of taps 0..2 on a
    side stream beside the encoder's later blocks (engine.hip dpt_fork, a
    parallel branch of the captured graph).  Only the launch order changes:
    the depth map must equal the one-stream forward bit for bit, in graph
    replay and eager mode."""
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 8)
    blob = pack.pack_bytes(sd, cfg, size, size)
    x = weights.synthetic_images(B, size, size, first_seed=31)
    os.environ["MDE_DPT_FORK"] = "1"
    try:
        y_fork = run_engine(blob, x, graph=True)
        y_fork_eager = run_engine(blob, x, graph=False)
        os.environ["MDE_DPT_FORK"] = "0"
        y_one = run_engine(blob, x, graph=True)
    finally:
        os.environ.pop("MDE_DPT_FORK", None)
    assert np.isfinite(y_one).all()
    assert np.array_equal(y_fork, y_one), "forked DPT branch (graph) must equal the one-stream forward"
    assert np.array_equal(y_fork_eager, y_one), "forked DPT branch (eager) must equal the one-stream forward"


@pytest.mark.parametrize("var,tile", [("MDE_GEMM_TILE", "big1"), ("MDE_GEMM_TILE", "128x128w8"),
                                      ("MDE_GEMM_W16", "1")])
def test_gemm_tile_variants_bit_exact(gpu, var, tile):
    """ViT-L 518^2 B=1 (config 3's unit) with the small-grid GEMM tilings
    (MDE_GEMM_TILE: tall 160/192-row tiles on a 3-deep ring, or 8 waves on
    the 128^2 tile, or 64 x 128 small-grid tiles; MDE_GEMM_W16: 16 waves of
    32 x 32 on the small-grid 128^2 tiles).  A tile's K loop runs in the same order whatever its
    shape and the split-K slicing is unchanged, so the depth map must equal
    the default tiling's bit for bit."""
    cfg = weights.model_config("vitl", "metric")
    sd = weights.synthetic_state_dict(cfg, 12)
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    x = weights.synthetic_images(1, 518, 518, first_seed=51)
    y_def = run_engine(blob, x)
    os.environ[var] = tile
    try:
        y_var = run_engine(blob, x)
    finally:
        os.environ.pop(var, None)
    assert np.isfinite(y_def).all()
    assert np.array_equal(y_var, y_def), f"{var}={tile} changed the result"


@pytest.mark.parametrize("encoder,head", [("vitl", "metric"), ("vitl", "relative")])
def test_gemm_stream_k(gpu, encoder, head):
    """ViT-L 518^2 B=1 (config 3's unit): qkv (264 tiles of 128^2), fc1 (352)
    and fc2 (88 tiles x 64 K-steps) under stream-K (gemm.hip gemm_sk_kernel):
    256 workgroups take whole tiles for as many full rounds as the grid holds,
    then equal shares of the remaining (tile, K-step) iterations; the last
    contributor of a cut tile sums the fp32 partial slots in contributor
    order.  Two runs (graph replay, then eager) must be bit-identical -- the
    order is fixed and every launch leaves its arrival counters at zero --
    and the map must match the whole-tile kernels (MDE_GEMM_SK=0) up to fp32
    reassociation, the same bar as the split-K test above.  Opt-in
    (MDE_GEMM_SK=1): measured slower than the whole-tile kernels."""
    cfg = weights.model_config(encoder, head)
    sd = weights.synthetic_state_dict(cfg, 14)
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    x = weights.synthetic_images(1, 518, 518, first_seed=61)
    y_tiles = run_engine(blob, x)
    os.environ["MDE_GEMM_SK"] = "1"  # opt-in (measured slower)
    try:
        y_sk = run_engine(blob, x, graph=True)
        assert np.isfinite(y_sk).all()
        assert np.array_equal(y_sk, run_engine(blob, x, graph=True)), "stream-K must be deterministic (graph replay)"
        assert np.array_equal(y_sk, run_engine(blob, x, graph=False)), "stream-K must be deterministic (eager)"
    finally:
        os.environ.pop("MDE_GEMM_SK", None)
    m = depth_metrics(y_sk, y_tiles)
    print(f"stream-K vs whole tiles {encoder} {head}", m)
    scale = float(np.abs(y_tiles).max())
    if head == "metric":  # 0.08 m of the 20 m range, as above
        assert m["max_abs"] < 0.004 * scale and m["rel_mean"] < 1.5e-3, m
    else:
        # the synthetic relative map is small (mean |y| ~ 1e-2), so the same
        # absolute noise is a larger fraction of it: measured rel_mean 3.8e-3,
        # max_abs 5.3e-3, corr 0.999993 (MI355X)
        assert m["rel_mean"] < 1e-2 and m["corr"] > 0.9999, m


@pytest.mark.parametrize("encoder", ["vits", "vitl"])
def test_fp32_precision_engine_vs_golden_518(gpu, encoder):
    """precision "fp32" (get_engine's reference default): the residual stream
    and every statistic stay fp32, MFMA operands f16 (a 10-bit mantissa, as
    the TF32 tensor-core path the reference's TensorRT fp32 build takes by
    default).  The default "fp16" engines above keep the stream in f16."""
    name = f"dav2_{encoder}_metric_518"
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    blob = pack.pack_bytes(sd, cfg, 518, 518, precision="fp32")
    x = weights.synthetic_images(1, 518, 518, first_seed=int(z["input_first_seed"]))
    y = run_engine(blob, x)
    check(y, z["output_hf_f16"].astype(np.float32), 20.0, f"{name} fp32-precision engine vs HF golden", encoder,
          extra_abs=F16_Q)

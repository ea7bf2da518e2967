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

from monocular_depth_estimation_trt_amd import _lib, pack, weights
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


@pytest.mark.parametrize("h,w,B", [(392, 518, 2), (672, 896, 1)])
def test_engine_reference_size_sweep_vs_oracle(gpu, h, w, B):
    """The reference's published size sweep (reports/tune/size_depth_anything_v2.json:
    392x518, 672x896; ViT-S metric, fp16 engines): upstream's bicubic pos-embed
    interpolation with the 0.1 offset (28 x 37 and 48 x 64 patch grids from the
    37 x 37 table; pinned by tests/golden/posembed_upstream.npz), 1037 / 3073
    tokens, every DPT size derived from the patch grid."""
    from oracle import dav2_ref
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 392 + w)
    x = weights.synthetic_images(B, h, w, first_seed=7)
    W = dav2_ref.to_torch(sd)
    ref = dav2_ref.forward(W, cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, h, w), x)
    assert y.shape == (B, h, w)
    # per-pixel bar derived from the attribution (VERDICT r05 item 3,
    # test_engine_worst_pixel_attribution): an IDEAL fp16 engine -- fp16
    # weights and fp16 storage where this engine stores fp16, fp32 arithmetic
    # otherwise -- is already 0.046 m from the fp32 oracle here (sigmoid *
    # 20 m at logits near 0); the engine may be up to 1.5x that, and never
    # held to less than the 0.3 %-of-max-depth bar
    import numerics_f16 as N
    e16 = float(np.abs(N.forward(W, cfg, x, N.STAGES)[0].numpy() - ref).max())
    extra = max(0.0, 1.5 * e16 - TOL["vits"][1] * 20.0)
    print(f"{h}x{w}: ideal-fp16 max |d| {e16:.4f} m -> max-abs bar {TOL['vits'][1] * 20.0 + extra:.4f} m")
    check(y, ref, 20.0, f"{h}x{w} B={B} vs oracle", extra_abs=extra)


@pytest.mark.parametrize("h,w,B", [(392, 518, 2), (672, 896, 1), (518, 518, 2)])
def test_engine_worst_pixel_attribution(gpu, h, w, B):
    """where the fp16 engine's largest per-pixel errors
    come from.  tests/numerics_f16.py reruns the fp32 oracle with fp16 STORAGE
    emulated at the engine's f16 storage points (residual stream, encoder
    operands, taps, DPT maps, head maps).  The metric head is
    sigmoid(logit) * 20 m, whose slope is 20 s (1 - s) ~ 5 m per logit unit
    near logit 0: a 0.01 logit error (f16 relative rounding is 4.9e-4) becomes
    ~0.05 m.  Measured at 392x518 (the reference's size, seed of
    test_engine_reference_size_sweep_vs_oracle): an ideal fp16 engine (fp16
    weights, fp16 storage at this engine's storage points, fp32 arithmetic
    otherwise) lands 0.046 m / rel_mean 4.1e-4 from the fp32 oracle (the
    residual stream's storage alone 0.039 m; tests/test_numerics_attribution.py),
    the engine 0.055 m / 4.3e-4 (round 6, profiles/r06_worst_pixel_attribution.log).
    Asserted here: the engine's worst pixel sits on the steep part of the
    sigmoid, and its error is within 1.5x of the ideal fp16 engine's -- the
    0.06 m bar's floor on these inputs is fp16 storage itself."""
    import numerics_f16 as N
    from oracle import dav2_ref
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = weights.model_config("vits", "metric")
    seed = 392 + w if (h, w) != (518, 518) else 910
    sd = weights.synthetic_state_dict(cfg, seed)
    x = weights.synthetic_images(B, h, w, first_seed=7)
    W = dav2_ref.to_torch(sd)
    ref = dav2_ref.forward(W, cfg, x).numpy()
    y16, _ = N.forward(W, cfg, x, N.STAGES)
    y16 = y16.numpy()
    _, logit = N.forward(W, cfg, x, ())
    logit = logit.numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, h, w), x)
    d_eng = np.abs(y - ref)
    d_sto = np.abs(y16 - ref)
    d_e16 = np.abs(y - y16)
    i = np.unravel_index(d_eng.argmax(), d_eng.shape)
    bar = TOL["vits"][1] * 20.0
    print(f"{h}x{w} B={B}: engine vs fp32 oracle max {d_eng.max():.4f} m at {tuple(int(v) for v in i)} "
          f"(logit {logit[i]:+.3f}, slope {20 * ref[i] / 20 * (1 - ref[i] / 20):.2f} m/unit); "
          f"f16-storage oracle vs fp32 max {d_sto.max():.4f}; engine vs f16-storage oracle max "
          f"{d_e16.max():.4f}; bar {bar:.3f} m, margin {bar - d_eng.max():.4f} m "
          f"({d_eng.max() / bar:.0%} of the bar)", flush=True)
    # the worst pixel is on the steep part of the sigmoid
    assert abs(logit[i]) < 1.5, logit[i]
    # fp16 storage explains the error scale: the engine is within 1.5x of it
    assert d_eng.max() <= 1.5 * d_sto.max() + 0.005, (d_eng.max(), d_sto.max())
    assert d_e16.max() <= 1.5 * d_sto.max() + 0.005, (d_e16.max(), d_sto.max())


def test_narrow_resid_matches_split(gpu):
    """Switch "narrow_resid" (gemm.hip): ViT-S 518^2 batch 1 runs fc2 and proj
    on 32 x 64 tiles with the whole K loop instead of split-K slices + the
    reduce launch.  Another fp32 association of the same sums: the two depth
    maps agree to fp16-storage noise (measured rel_mean 5.5e-4, max 0.040 m),
    and the narrow path meets the oracle bars."""
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 77)
    x = weights.synthetic_images(1, 518, 518, first_seed=5)
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    with _lib.tuning(narrow_resid=0):
        y0 = run_engine(blob, x)
    with _lib.tuning(narrow_resid=1):
        y1 = run_engine(blob, x)
    m = depth_metrics(y1, y0)
    print("narrow vs split", m)
    # two fp32 associations, each ~4e-4 (rel_mean) from the fp32 oracle by
    # fp16 storage (test_numerics_attribution): their difference is that
    # noise twice over, not a bias
    assert m["rel_mean"] < 1.2e-3 and m["max_abs"] < 0.08 and m["corr"] > 0.99999, m
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    check(y1, ref, 20.0, "narrow_resid B=1 vs oracle")


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
    config 3's B=1); the slices are summed in order, so the result is
    deterministic and equal to the unsplit GEMM (switch "splitk" = 0) up to
    fp32 reassociation."""
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 5)
    blob = pack.pack_bytes(sd, cfg, size, size)
    x = weights.synthetic_images(1, size, size, first_seed=21)
    y_split = run_engine(blob, x, graph=True)
    assert np.array_equal(y_split, run_engine(blob, x, graph=False)), "split-K must be deterministic"
    with _lib.tuning(splitk=0):
        y_plain = run_engine(blob, x)
    m = depth_metrics(y_split, y_plain)
    print(f"split-K vs unsplit {encoder} {size}", m)
    # the fp32 reassociation is amplified by the downstream f16 roundings
    # (measured ViT-S 0.026 m / 6.6e-4, ViT-L 0.036 m / 6.2e-4)
    assert m["max_abs"] < 0.08 and m["rel_mean"] < 1.5e-3, m


@pytest.mark.parametrize("encoder,size,B", [("vits", 518, 1), ("vits", 518, 8), ("vitl", 518, 1), ("vits", 98, 2),
                                            ("vitb", 126, 1)])
def test_resize_fold_bit_exact(gpu, encoder, size, B):
    """Switch "resize_fold" (engine.hip dav2_fusion, GemmParams::res1_up): the
    fusion blocks' x2 resize is not launched; the next block's rcu1 second conv
    reads the 1x1 output through the same align_corners blend (mde_device.h
    upsample8) in its epilogue -- the direct conv -- or writes it into the
    buffer first where its route is another kernel (the persistent 64-channel
    conv at B = 8, split-K at ViT-L B = 1's 37^2 / 74^2).  The same f16
    values reach the same adds: the depth map is bit-identical."""
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 41)
    blob = pack.pack_bytes(sd, cfg, size, size)
    x = weights.synthetic_images(B, size, size, first_seed=13)
    with _lib.tuning(resize_fold=1):
        y_fold = run_engine(blob, x)
    with _lib.tuning(resize_fold=0):
        y_plain = run_engine(blob, x)
    assert np.isfinite(y_fold).all()
    assert np.array_equal(y_fold, y_plain), depth_metrics(y_fold, y_plain)


@pytest.mark.parametrize("encoder,size", [("vitl", 518), ("vits", 98)])
def test_splitk_fused_matches_two_kernel(gpu, encoder, size):
    """Switch "splitk_fused" (gemm.hip gemm_kernel SPLIT): the engines' split-K
    GEMMs -- fc2 (E_RESID, ViT-L B=1: 88 128^2 tiles x 4 slices; ViT-S 98^2:
    64^2 tiles) and the DPT's split convs (E_STORE) -- run as ONE launch whose
    last-arriving slice per tile adds the slots in slice order, instead of the
    slices + splitk_resid / splitk_store.  The slice sums are the same fp32
    additions in the same order; only the folded-LN partials of the fc2 rows
    are grouped differently (8 columns per lane instead of 4), so the depth
    maps agree to f16 noise, replays are bit-identical (the arrival counters
    are re-zeroed by every launch) and the fused path meets the oracle bars.
    Off by default: its slots and counters go through system-scope accesses
    (the slices of a tile sit on different XCDs), and those round trips cost
    more than the reduce launch they replace (ViT-L B=1 3.17 -> 3.79 ms,
    gpurun_out r6f1)."""
    from oracle import dav2_ref
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 31)
    blob = pack.pack_bytes(sd, cfg, size, size)
    x = weights.synthetic_images(1, size, size, first_seed=71)
    with _lib.tuning(splitk_fused=1):
        y_fused = run_engine(blob, x, graph=True)
        assert np.array_equal(y_fused, run_engine(blob, x, graph=False)), "fused split-K must be deterministic"
        assert np.array_equal(y_fused, run_engine(blob, x, graph=True)), "a second context must see zeroed counters"
    with _lib.tuning(splitk_fused=0):
        y_two = run_engine(blob, x)
    m = depth_metrics(y_fused, y_two)
    print(f"fused vs two-kernel split-K {encoder} {size}", m)
    assert m["rel_mean"] < 1e-3 and m["max_abs"] < 0.08 and m["corr"] > 0.99999, m
    if encoder == "vits":
        ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
        check(y_fused, ref, 20.0, f"fused split-K {encoder} {size} vs oracle")


@pytest.mark.parametrize("switch", ["deep64", "w8small"])
def test_gemm_small_grid_variants_bit_exact(gpu, switch):
    """ViT-L 518^2 B=1 (config 3's unit) with a small-grid GEMM tiling switched
    off (tuning.h: "deep64" = the 4-deep ring of the 64^2 tiles and split-K
    slices, "w8small" = 8 waves on the 128^2 tiles of qkv / fc1 / the fc2
    slices).  A tile's K loop runs in the same order whatever its ring depth or
    wave count and the split-K slicing does not depend on either switch, so
    the depth map must equal the default tiling's bit for bit."""
    cfg = weights.model_config("vitl", "metric")
    sd = weights.synthetic_state_dict(cfg, 12)
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    x = weights.synthetic_images(1, 518, 518, first_seed=51)
    y_def = run_engine(blob, x)
    with _lib.tuning(**{switch: 0}):
        y_var = run_engine(blob, x)
    assert np.isfinite(y_def).all()
    assert np.array_equal(y_var, y_def), f"{switch}=0 changed the result"


def _oracle_chunks(sd, cfg, x, chunk=8):
    from oracle import dav2_ref
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    w = dav2_ref.to_torch(sd)
    return np.concatenate([dav2_ref.forward(w, cfg, x[i:i + chunk]).numpy() for i in range(0, len(x), chunk)])


@pytest.mark.parametrize("B", [32, 48])
def test_engine_518_bench_batches_vs_oracle(gpu, B):
    """The graphs the bench times (bench.py: ViT-S 518^2, B = 48 per GPU, a
    context sized for exactly that batch, hipGraph replay): B = 48 runs the
    8-wave 256-query attention (g256 = 6 x 48 x 6 >= 512) and the 256 x 128
    8-wave residual tiles (t256 >= 512 from B = 32 on), which the B <= 8 tests
    above never reach.  B = 32 is the first batch on the 256 x 128 residual
    tiles.  Every map against the fp32 oracle at the DA-V2 bars
    (verify_accuracy.py:54-55 thresholds are far looser)."""
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)   # the bench's weights
    x = weights.synthetic_images(B, 518, 518, first_seed=0)
    y = run_engine(pack.pack_bytes(sd, cfg, 518, 518), x)
    ref = _oracle_chunks(sd, cfg, x)
    assert y.shape == (B, 518, 518)
    check(y, ref, 20.0, f"518 B={B} (bench graph) vs oracle")
    worst = max(depth_metrics(y[i:i + 1], ref[i:i + 1])["max_abs"] for i in range(B))
    assert worst <= 0.003 * 20.0, worst


def test_engine_b48_replays_bit_identical(gpu):
    """The bench's graph (ViT-S 518^2, B = 48) replayed three times in one
    context and once eagerly gives bit-identical maps: every kernel on the
    path is deterministic (no atomics, fixed split-K / key-group merge
    orders) and no LDS-DMA races its consumers -- round 4's fused-MLP
    experiment lost exactly this property to an address-register race
    (DESIGN.md section 9), so it is checked on the product graph."""
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    B = 48
    x = weights.synthetic_images(B, 518, 518, first_seed=3)
    eng = Engine.from_bytes(pack.pack_bytes(sd, cfg, 518, 518), 0,
                            profile=((1, 3, 518, 518), (B, 3, 518, 518), (B, 3, 518, 518)))
    ctx = eng.create_execution_context()
    xin = torch.from_numpy(x).cuda()
    out = torch.empty(B, 518, 518, device="cuda")
    ctx.set_input_shape("input", x.shape)
    ctx.set_tensor_address("input", xin.data_ptr())
    ctx.set_tensor_address("output", out.data_ptr())
    ys = []
    for graph in (True, True, True, False):
        ctx.set_graph_mode(graph)
        out.fill_(float("nan"))
        ctx.execute_async_v3(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ys.append(out.cpu().numpy())
    ctx.destroy()
    eng.destroy()
    assert np.isfinite(ys[0]).all()
    for i, y in enumerate(ys[1:], 1):
        assert np.array_equal(y, ys[0]), f"run {i} differs: max {np.abs(y - ys[0]).max()}"


def test_lnfold_matches_layernorm(gpu):
    """Switch "lnfold" = 0 (read at context creation): norm1 / norm2 / the tap
    norms as LayerNorm launches and the unfolded qkv / fc1 / project weights,
    against the default folded engine -- both within the DA-V2 bars of the
    oracle, and close to each other (one more f16 rounding of the normed
    rows on the unfolded side)."""
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 808)
    x = weights.synthetic_images(2, 518, 518, first_seed=70)
    blob = pack.pack_bytes(sd, cfg, 518, 518)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y_fold = run_engine(blob, x)
    with _lib.tuning(lnfold=0):
        y_ln = run_engine(blob, x)
    check(y_fold, ref, 20.0, "518 B=2 folded LN vs oracle")
    check(y_ln, ref, 20.0, "518 B=2 LayerNorm launches vs oracle")
    m = depth_metrics(y_fold, y_ln)
    print("folded vs unfolded LN", m)
    assert m["rel_mean"] < 1.5e-3 and m["corr"] >= CORR, m


def test_enqueue_inside_caller_capture(gpu):
    """A caller that captures its own stream (torch.cuda.graph) gets the
    forward's kernels captured into its graph (engine.hip: no graph of ours
    is launched inside a capture); replaying the caller's graph on new input
    equals the engine's own result, and more distinct shapes than the
    context's graph cache holds can go through it."""
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 5)
    blob = pack.pack_bytes(sd, cfg, 98, 98)
    xa = weights.synthetic_images(3, 98, 98, first_seed=90)
    xb = weights.synthetic_images(3, 98, 98, first_seed=93)
    ref_b = run_engine(blob, xb)
    eng = Engine.from_bytes(blob, 0, profile=((1, 3, 98, 98), (3, 3, 98, 98), (3, 3, 98, 98)))
    ctx = eng.create_execution_context()
    xin = torch.from_numpy(xa).cuda()
    out = torch.empty(3, 98, 98, device="cuda")
    ctx.set_input_shape("input", xa.shape)
    ctx.set_tensor_address("input", xin.data_ptr())
    ctx.set_tensor_address("output", out.data_ptr())
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ctx.execute_async_v3(s.cuda_stream)   # warm (eager outside capture: graph mode, own cache)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        ctx.execute_async_v3(s.cuda_stream)
    xin.copy_(torch.from_numpy(xb))
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref_b), "captured forward must equal the engine's own"
    # more (batch, address) keys than the context caches (kMaxGraphs = 8), all
    # captured into caller graphs
    graphs = []
    for i in range(10):
        o = torch.empty(3, 98, 98, device="cuda")
        ctx.set_tensor_address("output", o.data_ptr())
        gi = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gi, stream=s):
            ctx.execute_async_v3(s.cuda_stream)
        graphs.append((gi, o))
    for gi, o in graphs:
        gi.replay()
    torch.cuda.synchronize()
    for gi, o in graphs:
        assert np.array_equal(o.cpu().numpy(), ref_b)
    ctx.destroy()
    eng.destroy()


@pytest.mark.parametrize("encoder", ["vits", "vitl"])
def test_fp32_precision_engine_vs_golden_518(gpu, encoder):
    """precision "fp32" (get_engine's reference default, core/common.py:141-144):
    the exact-fp32 engine (fp32.hip: fp32 weights and activations through the
    encoder AND the DPT head, fp32 MFMA) against the full-map HF golden,
    whose f16 storage is then the only visible error."""
    name = f"dav2_{encoder}_metric_518"
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, int(z["seed"]))
    blob = pack.pack_bytes(sd, cfg, 518, 518, precision="fp32")
    x = weights.synthetic_images(1, 518, 518, first_seed=int(z["input_first_seed"]))
    y = run_engine(blob, x)
    m = check(y, z["output_hf_f16"].astype(np.float32), 20.0, f"{name} exact-fp32 encoder vs HF golden", encoder,
              extra_abs=F16_Q)
    # against the f16-stored golden: the storage rounding (<= 2^-11 relative)
    # is all that should remain (measured 1.77e-4 / 1.72e-4 for ViT-S / ViT-L;
    # the f16 head left 6.07e-4 at ViT-S in round 4)
    assert m["rel_mean"] <= 3e-4, m


@pytest.mark.parametrize("encoder,B", [("vits", 2), ("vitl", 1)])
def test_fp32_precision_engine_vs_oracle_98(gpu, encoder, B):
    """The exact-fp32 engine at 98^2 (both grid forms of the fp32 GEMM and
    attention) against the fp32 oracle: every layer fp32 on both sides, so
    what remains is summation order and v_exp_f32 (fp32 rounding level) --
    the pin that an f16 operand anywhere in the engine would break."""
    from oracle import dav2_ref
    cfg = weights.model_config(encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 31)
    x = weights.synthetic_images(B, 98, 98, first_seed=7)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y = run_engine(pack.pack_bytes(sd, cfg, 98, 98, precision="fp32"), x)
    m = check(y, ref, 20.0, f"{encoder} 98 B={B} exact-fp32 vs oracle", encoder)
    # measured (MI355X, round 5): ViT-S rel_mean 6.1e-7 / max 3.9e-5 m, ViT-L
    # 1.2e-6 / 4.1e-5 m -- fp32 rounding; the bars are ~5x that
    assert m["rel_mean"] <= 5e-6 and m["max_abs"] <= 2e-4, m


def test_fp32_precision_range_beyond_f16(gpu):
    """Range: block 5's MLP hidden layer scaled by 2e5 (fc1 weights and bias x
    2e5, fc2 weights / 2e5 -- the same function in real arithmetic, hidden
    activations ~1e5, past f16's 65504).  The exact-fp32 engine follows the
    oracle; the fp16 engine's f16 hidden layer overflows there (reported, the
    reason the reference's default build is fp32 TensorRT)."""
    from oracle import dav2_ref
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 44)
    s = 2e5
    k = "pretrained.blocks.5.mlp."
    sd[k + "fc1.weight"] = sd[k + "fc1.weight"] * s
    sd[k + "fc1.bias"] = sd[k + "fc1.bias"] * s
    sd[k + "fc2.weight"] = sd[k + "fc2.weight"] / s
    x = weights.synthetic_images(1, 98, 98, first_seed=17)
    ref = dav2_ref.forward(dav2_ref.to_torch(sd), cfg, x).numpy()
    y32 = run_engine(pack.pack_bytes(sd, cfg, 98, 98, precision="fp32"), x)
    y16 = run_engine(pack.pack_bytes(sd, cfg, 98, 98, precision="fp16"), x)
    finite16 = bool(np.isfinite(y16).all())
    with np.errstate(invalid="ignore", divide="ignore"):  # a collapsed (constant) map has no correlation
        m16 = depth_metrics(np.nan_to_num(y16, nan=0.0, posinf=0.0, neginf=0.0), ref)
    print("fp16 engine on the scaled model: finite", finite16, m16)
    # the scaling must really leave the f16 range, or the fp32 check below proves nothing
    assert (not finite16) or m16["rel_mean"] > 0.05, f"fp16 engine unaffected by the scaled hidden layer: {m16}"
    check(y32, ref, 20.0, "exact-fp32 engine, hidden layer past the f16 range")

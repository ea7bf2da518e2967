"""Where the fp16 engine's largest per-pixel errors come from (VERDICT r05
item 3), on the CPU: the fp32 oracle rerun with fp16 storage emulated at the
engine's f16 storage points and fp16 weights (tests/numerics_f16.py).

The metric head is sigmoid(logit) * max_depth (20 m).  With the synthetic
weights the logits sit near 0 (median |logit| ~1, depths ~5-15 m), where the
slope 20 * s * (1 - s) is 4-5 m per logit unit: fp16 rounding of O(5e-4) relative
upstream becomes a ~0.01 logit error and ~0.05 m.  At the reference's
392x518 size (the input of test_engine_reference_size_sweep_vs_oracle) an
IDEAL fp16 engine -- fp16 weights and fp16 storage exactly where this engine
stores fp16, fp32 arithmetic otherwise -- lands at rel_mean 4.1e-4 and max
|d| 0.046 m from the fp32 oracle; the residual stream's fp16 storage alone
gives 0.039 m.  The HIP engine measures rel_mean 4.3e-4, max 0.055 m
(tests/test_gpu_engine.py::test_engine_worst_pixel_attribution prints both
sides on the GPU box).  The 0.06 m bar (0.3 % of max_depth) therefore has a
floor of ~0.045 m set by fp16 storage itself on these inputs, not by a
kernel's summation order.
"""
import os

import numpy as np
import pytest
import torch

import numerics_f16 as N
from monocular_depth_estimation_trt_amd import weights
from oracle import dav2_ref


@pytest.fixture(scope="module")
def case():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    h, w, B = 392, 518, 2
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 392 + w)
    x = weights.synthetic_images(B, h, w, first_seed=7)
    W = dav2_ref.to_torch(sd)
    return cfg, W, x, dav2_ref.forward(W, cfg, x).numpy()


def _err(y, ref):
    d = np.abs(y - ref)
    return float(d.max()), float(d.mean() / np.abs(ref).mean())


def test_restated_forward_is_the_oracle(case):
    cfg, W, x, ref = case
    y, _ = N.forward(W, cfg, x, ())
    assert np.abs(y.numpy() - ref).max() < 1e-4


def test_ideal_fp16_engine_error_floor(case):
    cfg, W, x, ref = case
    mx_all, rel_all = _err(N.forward(W, cfg, x, N.STAGES)[0].numpy(), ref)
    mx_res, _ = _err(N.forward(W, cfg, x, ("resid",))[0].numpy(), ref)
    print(f"ideal fp16 engine: max {mx_all:.4f} m rel_mean {rel_all:.2e}; residual storage alone max {mx_res:.4f} m")
    # the storage floor is most of the 0.06 m bar on this input
    assert 0.03 <= mx_all <= 0.06 and 2e-4 <= rel_all <= 6e-4, (mx_all, rel_all)
    assert 0.025 <= mx_res <= 0.05, mx_res
    # ... and sits on the sigmoid's steep part: logits near 0 everywhere
    _, logit = N.forward(W, cfg, x, ())
    assert float(np.median(np.abs(logit.numpy()))) < 1.5

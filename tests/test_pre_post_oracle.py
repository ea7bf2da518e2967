"""The pre/post-process oracle (oracle/pre_post.py) against the reference's
own check of the uint8 preamble (tests/test_uint8_input.py:78-99: seed-0
8x8 uint8 image, host arithmetic vs preamble, max rel diff < 1e-6) and
against the properties of align_corners bilinear resizing."""

import os
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, ROOT)
from oracle import pre_post  # noqa: E402


def test_preamble_is_the_reference_host_arithmetic():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(1, 8, 8, 3), dtype=np.uint8)
    f = img.astype(np.float32) / 255.0
    f = (f - np.array(pre_post.MEAN, dtype=np.float32)) / np.array(pre_post.STD, dtype=np.float32)
    ref = np.ascontiguousarray(f.transpose(0, 3, 1, 2))
    got = pre_post.uint8_preamble(img)
    assert got.dtype == np.float32 and got.shape == (1, 3, 8, 8)
    assert np.array_equal(got, ref)


def test_preamble_matches_float64_normalisation_to_f32_rounding():
    from monocular_depth_estimation_trt_amd import weights
    u = weights.synthetic_images_u8(1, 28, 42, first_seed=3)
    x64 = weights.synthetic_images(1, 28, 42, first_seed=3)
    assert np.abs(pre_post.uint8_preamble(u) - x64).max() <= 2e-6


def test_postprocess_corners_and_clamp():
    d = np.array([[[0.0, 1.0], [2.0, 5000.0]]], np.float32)
    y = pre_post.postprocess(d, 3, 5)
    assert y.shape == (1, 3, 5)
    # align_corners=True: corners are the source corners (then clamped)
    assert y[0, 0, 0] == np.float32(1e-3) and y[0, 0, -1] == 1.0 and y[0, -1, 0] == 2.0 and y[0, -1, -1] == 1e3
    assert abs(y[0, 0, 2] - 0.5) < 1e-6


def test_patch_matrix_layout():
    x = np.arange(1 * 3 * 28 * 28, dtype=np.float32).reshape(1, 3, 28, 28) % 97
    P = pre_post.patch_matrix(x)
    assert P.shape == (4, 672)
    # patch (py=1, px=0), channel 2, kernel row 3, column 5
    assert P[2, 2 * 224 + 3 * 16 + 5] == np.float16(x[0, 2, 14 + 3, 5])
    assert (P.reshape(4, 3, 14, 16)[..., 14:] == 0).all()

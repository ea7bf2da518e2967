"""VGGT host side, CPU only: the oracle against the committed golden vectors
(the reference's own export patches and transformers' Dinov2WithRegisters,
tests/golden/make_golden_vggt.py), the packer's folds and tables against the
oracle, the config record, and oracle properties (tests/test_gpu_vggt.py
holds the engine parity tests)."""

import os
import struct

import numpy as np
import torch
import torch.nn.functional as F

from conftest import GOLDEN
from monocular_depth_estimation_trt_amd import flops_vggt, pack_vggt as PV, weights_vggt as WV
from oracle import vggt_ref


def _golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_positions_match_reference_export_patch():
    z = _golden("vggt_export_compat.npz")
    for h, w in ((37, 37), (7, 7), (5, 9)):
        ref = z[f"pos_{h}x{w}"]
        assert ref.shape == (2, h * w, 2)
        assert np.array_equal(vggt_ref.position_grid(h, w).numpy(), ref[0])


def test_sincos_matches_reference_export_patch():
    z = _golden("vggt_export_compat.npz")
    coords = vggt_ref.create_uv_grid(37, 37, 1.0).reshape(-1, 2)
    np.testing.assert_allclose(coords.numpy(), z["uv_37"], atol=1e-7)
    for dim in (64, 128):
        for axis in (0, 1):
            got = vggt_ref.make_sincos_pos_embed(dim // 2, coords[:, axis], 100).numpy()
            np.testing.assert_allclose(got, z[f"sincos_{dim}_{axis}"], atol=1e-6)


def test_dino_encoder_matches_hf_golden():
    z = _golden("vggt_dino_tiny.npz")
    cfg = WV.vggt_config("tiny")
    sd = WV.synthetic_state_dict(cfg, int(z["seed"]))
    assert WV.state_dict_digest(sd) == str(z["weights_sha256"]), "weight generator drifted"
    got = vggt_ref.dinov2_reg(vggt_ref.to_torch(sd), cfg, torch.from_numpy(z["input_norm"])).numpy()
    np.testing.assert_allclose(got, z["tokens_hf"], atol=1e-4, rtol=1e-4)


def test_uv_embed_packer_equals_oracle():
    for C, n in ((32, 7), (256, 37), (128, 98)):
        got = PV.uv_embed(C, n, n, 1.0)                                     # [n*n, C] float64
        ref = vggt_ref.uv_embed(C, n, n, 1.0).permute(1, 2, 0).reshape(n * n, C).double().numpy()
        np.testing.assert_allclose(got, ref, atol=2e-6)


def test_rope_tables_equal_oracle():
    cos, sin = PV.rope_tables(39)
    rc, rs = vggt_ref.rope_tables(32, 39)
    np.testing.assert_allclose(cos, rc[:, :16].numpy(), atol=1e-5)
    np.testing.assert_allclose(sin, rs[:, :16].numpy(), atol=1e-5)
    assert torch.equal(rc[:, :16], rc[:, 16:])     # duplicated angles: the kernel reads one half


def test_patch_embed_fold_exact():
    rng = np.random.default_rng(0)
    w = rng.standard_normal((16, 3, 14, 14)).astype(np.float32)
    b = rng.standard_normal(16).astype(np.float32)
    x = rng.random((2, 3, 28, 42))
    mean = np.asarray(WV.RESNET_MEAN)[None, :, None, None]
    std = np.asarray(WV.RESNET_STD)[None, :, None, None]
    ref = F.conv2d(torch.from_numpy((x - mean) / std), torch.from_numpy(w.astype(np.float64)),
                   torch.from_numpy(b.astype(np.float64)), stride=14)
    wf, bf = PV.fold_patch_embed(w, b)
    got = F.conv2d(torch.from_numpy(x), torch.from_numpy(wf.astype(np.float64)),
                   torch.from_numpy(bf.astype(np.float64)), stride=14)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=5e-5)


def test_head_pe_is_conv_of_embedding():
    """conv(x + pe) == conv(x) + head_pe: the fold the head epilogue relies on."""
    rng = np.random.default_rng(1)
    w = (rng.standard_normal((32, 16, 3, 3)) * 0.1).astype(np.float32)
    n = 11
    x = torch.from_numpy(rng.standard_normal((1, 16, n, n)))
    pe = vggt_ref.uv_embed(16, n, n, 1.0).double()[None]
    wt = torch.from_numpy(w.astype(np.float64))
    ref = F.conv2d(x + pe, wt, padding=1)
    got = F.conv2d(x, wt, padding=1) + torch.from_numpy(PV.head_pe(w, n, n)).T.reshape(1, 32, n, n)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), atol=1e-5)


def _unpack(blob):
    n = struct.unpack_from("<I", blob, 12)[0]
    cfg = blob[32:32 + 256]
    tensors = {}
    for i in range(n):
        name, dt, nd, d0, d1, d2, d3, off, nb, _ = struct.unpack_from("<80sii4iQQ8s", blob, 288 + 128 * i)
        tensors[name.rstrip(b"\0").decode()] = (dt, [d0, d1, d2, d3][:nd], off, nb)
    return cfg, tensors


def test_pack_config_and_tensors():
    cfg = WV.vggt_config("tiny")
    sd = WV.synthetic_state_dict(cfg, 2468)
    blob = PV.pack_bytes(sd, cfg, frames=2)
    c, t = _unpack(blob)
    assert struct.unpack_from("<8i", c, 0) == (128, 2, 2, 512, 14, 98, 98, 64)
    assert struct.unpack_from("<4i", c, 48) == (0, 1, 2, 3)                  # taps
    assert struct.unpack_from("<2i", c, 64) == (32, 2)                       # head_hidden, metric = exp head
    assert struct.unpack_from("<i", c, 128)[0] == PV.FAMILY_VGGT
    assert struct.unpack_from("<3i", c, 180) == (2, 5, 4)                    # frames, npre, aa_depth
    assert abs(struct.unpack_from("<f", c, 192)[0] - 1e-5) < 1e-10
    assert t["patch.w"][1] == [128, 704] and t["pos.patch"][1] == [49, 128]  # K 672 padded to x64
    assert t["pre.dino"][1] == [5, 128] and t["pre.agg"][1] == [2, 5, 128]
    assert t["fb3.qn.g"][1] == [64] and t["gb0.qkv.w"][1] == [384, 128] and "db0.qn.g" not in t
    assert t["proj2.w"][1] == [128, 256] and t["pe2"][1] == [49, 128] and t["pe2"][0] == 1
    assert t["head.pe"][1] == [98 * 98, 32] and t["head.c3.w"][1] == [32] and t["head.c3.b"][1] == [1]
    assert "rf4.rcu1.c1.w" not in t and "rf3.rcu1.c1.w" in t
    assert t["rope.cos"][1][1] == 16 and t["rope.cos"][1][0] >= 8


def test_rcu_skip_adds_relu_input():
    """In-place ReLU semantics: with zero conv weights a unit returns relu(x)."""
    Fc = 4
    w = {"u.conv1.weight": torch.zeros(Fc, Fc, 3, 3), "u.conv1.bias": torch.zeros(Fc),
         "u.conv2.weight": torch.zeros(Fc, Fc, 3, 3), "u.conv2.bias": torch.zeros(Fc)}
    x = torch.randn(1, Fc, 5, 5)
    assert torch.equal(vggt_ref._rcu(w, "u.", x), F.relu(x))


def test_tiny_oracle_is_input_dependent_and_multi_frame():
    cfg = WV.vggt_config("tiny")
    w = vggt_ref.to_torch(WV.synthetic_state_dict(cfg, 2468))
    x = WV.synthetic_images(1, 2, cfg["img"], first_seed=5)
    y2 = vggt_ref.forward(w, cfg, x)
    assert y2.shape == (1, 2, 98, 98, 1) and bool(torch.isfinite(y2).all()) and float(y2.min()) > 0
    y1 = vggt_ref.forward(w, cfg, x[:, :1])
    # frame 0 sees frame 1 through global attention: the pair differs from the single frame
    assert float((y2[:, 0] - y1[:, 0]).abs().max()) > 1e-4
    yb = vggt_ref.forward(w, cfg, x[:, 1:])
    assert float((y2[:, 1] - yb[:, 0]).abs().max()) > 1e-4


def test_vggt_1b_parameter_count_and_flops():
    cfg = WV.vggt_config("vggt_1b")
    n = sum(int(np.prod(s)) for s in WV.expected_shapes(cfg).values())
    assert 0.9e9 < n < 1.0e9, n          # the depth path of VGGT-1B (no camera / point / track heads)
    gf = flops_vggt.total_flops(cfg) / 1e9
    assert 3200 < gf < 3500, gf
    assert flops_vggt.layer_class("gb17.attn") == "gb.attn"
    assert flops_vggt.layer_class("rf3.rcu1.c2") == "rcu.conv"


def test_get_engine_recognises_vggt_sources():
    from monocular_depth_estimation_trt_amd import common
    assert common.is_vggt_source("synthetic:vggt:tiny")
    assert not common.is_vggt_source("synthetic:vits")
    cfg = WV.vggt_config("tiny")
    sd = WV.synthetic_state_dict(cfg, 1)
    assert common.is_vggt_source("/x/model.pt", sd)
    assert common._vggt_config_of(sd)["encoder"] == "tiny"

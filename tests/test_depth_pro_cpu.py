"""Depth Pro host side, CPU only: the synthetic checkpoint layout against
transformers' DepthProForDepthEstimation, the oracle against the committed
HF golden (tests/golden/make_golden_depth_pro.py), and the packer (config
record, tensor layouts, the deconv + projection fold)."""

import os
import struct

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN
from monocular_depth_estimation_trt_amd import pack_depth_pro as PD
from monocular_depth_estimation_trt_amd import weights_depth_pro as WD
from oracle import depth_pro_ref


@pytest.mark.parametrize("preset", ["tiny", "dinov2l16_384"])
def test_synthetic_layout_matches_hf(preset):
    """Key names and shapes == transformers' DepthProForDepthEstimation built
    from the equivalent local config (meta device: no memory, no weights)."""
    tf = pytest.importorskip("transformers")
    import importlib.util
    spec = importlib.util.spec_from_file_location("mgdp", os.path.join(GOLDEN, "make_golden_depth_pro.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    cfg = WD.depth_pro_config(preset)
    with torch.device("meta"):
        m = tf.DepthProForDepthEstimation(mg.hf_config(cfg))
    hf = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert hf == WD.expected_shapes(cfg)


def test_oracle_matches_hf_golden():
    z = np.load(os.path.join(GOLDEN, "depth_pro_tiny_b2.npz"), allow_pickle=False)
    cfg = WD.depth_pro_config(str(z["preset"]), use_fov=bool(int(z["use_fov"])))
    sd = WD.synthetic_state_dict(cfg, int(z["seed"]))
    assert WD.state_dict_digest(sd) == str(z["weights_sha256"]), "weight generator drifted"
    x = WD.synthetic_images(int(z["batch"]), cfg["img"], first_seed=int(z["input_first_seed"]))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    y, fov = depth_pro_ref.forward(depth_pro_ref.to_torch(sd), cfg, x)
    y = y.numpy()
    np.testing.assert_allclose(y[:, ::8, ::8], z["output_hf_sub8"], atol=2e-4, rtol=1e-4)
    assert abs(float(y.mean()) - float(z["out_mean"])) < 1e-4
    np.testing.assert_allclose(fov.numpy(), z["fov_hf"], atol=1e-5, rtol=1e-5)


def test_oracle_matches_hf_golden_real_widths():
    """The "dinov2l16_384_shallow" preset: the real Depth Pro widths (D 1024,
    16 heads, decoder 256, scaled dims 1024/1024/512), 4 blocks per encoder,
    B=1 at 1536^2 -- the full-width fixture the GPU test checks the engine on."""
    z = np.load(os.path.join(GOLDEN, "depth_pro_shallow_b1.npz"), allow_pickle=False)
    cfg = WD.depth_pro_config(str(z["preset"]), use_fov=bool(int(z["use_fov"])))
    assert (cfg["embed_dim"], cfg["num_heads"], cfg["fusion"], cfg["scaled_dims"]) == (1024, 16, 256, [1024, 1024, 512])
    sd = WD.synthetic_state_dict(cfg, int(z["seed"]))
    assert WD.state_dict_digest(sd) == str(z["weights_sha256"]), "weight generator drifted"
    x = WD.synthetic_images(1, cfg["img"], first_seed=int(z["input_first_seed"]))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    y, fov = depth_pro_ref.forward(depth_pro_ref.to_torch(sd), cfg, x)
    ref = z["output_hf_sub2_f16"].astype(np.float32)
    np.testing.assert_allclose(y.numpy()[:, ::2, ::2], ref, atol=1e-2, rtol=1e-3)   # f16 storage
    assert abs(float(y.mean()) - float(z["out_mean"])) < 1e-4
    np.testing.assert_allclose(fov.numpy(), z["fov_hf"], atol=1e-5, rtol=1e-5)


def test_merge_geometry():
    """The 1536 geometry: every merged level comes out at its target size, so
    HF's bilinear resize after the merge is the identity."""
    for img, vit, ratio, ov, pad, want in ((1536, 384, 1.0, 0.25, 3, 96), (1536, 384, 0.5, 0.5, 6, 48),
                                           (1536, 384, 0.25, 0.0, 12, 24)):
        s, n, stride = depth_pro_ref.patch_grid(img, vit, ratio, ov)
        G = 24
        maps = torch.zeros(n * n, 1, G, G)
        assert depth_pro_ref.merge(maps, 1, pad).shape[-1] == want


def _unpack(blob):
    n = struct.unpack_from("<I", blob, 12)[0]
    cfg = blob[32:32 + 256]
    tensors = {}
    for i in range(n):
        name, dt, nd, d0, d1, d2, d3, off, nb, _ = struct.unpack_from("<80sii4iQQ8s", blob, 288 + 128 * i)
        tensors[name.rstrip(b"\0").decode()] = (dt, [d0, d1, d2, d3][:nd], off, nb)
    return cfg, tensors


def test_pack_config_and_tensors():
    cfg = WD.depth_pro_config("tiny")
    sd = WD.synthetic_state_dict(cfg, 4321)
    blob = PD.pack_bytes(sd, cfg)
    c, t = _unpack(blob)
    ints = struct.unpack_from("<8i", c, 0)
    assert ints[:8] == (128, 4, 2, 512, 16, 1536, 1536, 128)
    fam = struct.unpack_from("<6i2i2i3i", c, 128)
    assert fam == (1, 384, 3, 1, 2, 6, 3, 1, 128, 128, 256, 256, 128)
    for p in ("pe.", "ie.", "fe."):
        assert t[p + "patch.w"][1] == [128, 768] and t[p + "pos.patch"][1] == [576, 128]
        assert t[p + "b3.qkv.w"][1] == [384, 128]
    assert t["fs0.up.w"][1] == [4 * 128, 128] and "fs0.rcu1.c1.w" not in t and "fs1.rcu1.c1.w" in t
    assert t["fov.final.w"][1] == [6 * 6 * 16] and "prj4.w" not in t   # inter_dims[1] == fusion: Identity


def test_deconv_projection_fold():
    torch.manual_seed(0)
    Fc = 16
    wt = torch.randn(Fc, Fc, 2, 2)
    wp = torch.randn(Fc, Fc, 1, 1)
    x = torch.randn(1, Fc, 5, 7)
    ref = F.conv2d(F.conv_transpose2d(x, wt, stride=2), wp)
    fw = torch.from_numpy(PD.fold_deconv_projection(wt.numpy(), wp.numpy()))
    got = F.conv_transpose2d(x, fw, stride=2)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_fov_final_layout():
    """fov.final.w is the 6x6 valid conv weight in the NHWC order of the map it dots with."""
    cfg = WD.depth_pro_config("tiny")
    sd = WD.synthetic_state_dict(cfg, 4321)
    w = sd["fov_model.head.layers.4.weight"]            # [1][C][6][6]
    tens = PD.packed_tensors(sd, cfg)
    z = np.random.default_rng(0).standard_normal((1, w.shape[1], 6, 6)).astype(np.float32)
    ref = float((w * z).sum())
    got = float(tens["fov.final.w"] @ z[0].transpose(1, 2, 0).reshape(-1))
    assert abs(got - ref) < 1e-4

"""AOT packer: file format, layouts (checked numerically against torch ops),
and the engine-build fingerprint.  CPU only."""

import struct

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from monocular_depth_estimation_trt_amd import pack, weights


@pytest.fixture(scope="module")
def small():
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 7)
    return cfg, sd


def parse(blob):
    magic, ver, n, doff, dbytes = struct.unpack_from("<8sIIQQ", blob, 0)
    cfgb = blob[32:32 + 256]
    ints = struct.unpack_from("<8i4i4i2i", cfgb, 0)
    md, eps = struct.unpack_from("<2f", cfgb, 72)
    tens = {}
    for i in range(n):
        name, dt, nd, d0, d1, d2, d3, off, nb, _ = struct.unpack_from("<80sii4iQQ8s", blob, 288 + 128 * i)
        shape = (d0, d1, d2, d3)[:nd]
        raw = blob[doff + off: doff + off + nb]
        tens[name.rstrip(b"\0").decode()] = np.frombuffer(raw, np.float32 if dt == 0 else np.float16).reshape(shape)
    return dict(magic=magic, version=ver, n=n, data_offset=doff, data_bytes=dbytes, ints=ints, max_depth=md,
                eps=eps), tens


def test_header_and_table(small):
    cfg, sd = small
    blob = pack.pack_bytes(sd, cfg, 98, 126)
    h, t = parse(blob)
    assert h["magic"] == b"MDEPACK1" and h["version"] == pack.PACK_VERSION
    assert h["data_offset"] % 256 == 0 and len(blob) == h["data_offset"] + h["data_bytes"]
    D, depth, heads, mlp, patch, img_h, img_w, F_ = h["ints"][:8]
    assert (D, depth, heads, mlp, patch, img_h, img_w, F_) == (384, 12, 6, 1536, 14, 98, 126, 64)
    assert list(h["ints"][8:12]) == [48, 96, 192, 384] and list(h["ints"][12:16]) == [2, 5, 8, 11]
    assert h["ints"][16:18] == (32, 1) and h["max_depth"] == 20.0
    assert abs(h["eps"] - 1e-6) < 1e-12
    assert t["pos.patch"].shape == (7 * 9, 384)
    for name, a in t.items():
        if a.dtype == np.float16 and a.ndim == 2:
            assert a.shape[0] % 128 == 0 and a.shape[1] % 64 == 0, name


def test_linear_layouts(small):
    cfg, sd = small
    _, t = parse(pack.pack_bytes(sd, cfg, 98, 98))
    w = sd["pretrained.blocks.3.mlp.fc1.weight"]
    np.testing.assert_array_equal(t["b3.fc1.w"][:1536, :384], w.astype(np.float16))
    assert not t["b3.fc1.w"][:, 384:].any()
    np.testing.assert_array_equal(t["b0.ls2"], sd["pretrained.blocks.0.ls2.gamma"])


def _conv_via_packed(wp, x, cin, cout, stride=1):
    """3x3 pad-1 conv computed from the packed [Cout][ky][kx][Cin] rows (im2col)."""
    B, _, H, W = x.shape
    cols = F.unfold(x, 3, padding=1, stride=stride)             # [B, Cin*9, L] in (ci, ky, kx) order
    cols = cols.reshape(B, cin, 9, -1).permute(0, 2, 1, 3).reshape(B, 9 * cin, -1)   # (ky, kx, ci)
    w = torch.from_numpy(wp[:cout, :9 * cin].astype(np.float32))
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    return (w @ cols).reshape(B, cout, Ho, Wo)


def test_conv3_layout_matches_torch(small):
    cfg, sd = small
    _, t = parse(pack.pack_bytes(sd, cfg, 98, 98))
    x = torch.randn(2, 96, 9, 11)
    w = torch.from_numpy(sd["depth_head.scratch.layer2_rn.weight"]).half().float()
    ref = F.conv2d(x, w, padding=1)
    got = _conv_via_packed(t["rn2.w"], x, 96, 64)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
    w3 = torch.from_numpy(sd["depth_head.resize_layers.3.weight"]).half().float()
    ref3 = F.conv2d(x.new_zeros(1, 384, 7, 7).normal_(), w3, stride=2, padding=1)
    assert ref3.shape == (1, 384, 4, 4)


def test_convT_layout_matches_torch(small):
    cfg, sd = small
    _, t = parse(pack.pack_bytes(sd, cfg, 98, 98))
    for idx, s, c in ((0, 4, 48), (1, 2, 96)):
        x = torch.randn(1, c, 5, 6)
        w = torch.from_numpy(sd[f"depth_head.resize_layers.{idx}.weight"]).half().float()
        ref = F.conv_transpose2d(x, w, stride=s)
        wp = torch.from_numpy(t[f"rs{idx}.w"][:s * s * c, :c].astype(np.float32))     # [(dy,dx,co)][ci]
        y = (x.permute(0, 2, 3, 1).reshape(-1, c) @ wp.T).reshape(1, 5, 6, s, s, c)  # [b,y,x,dy,dx,co]
        got = y.permute(0, 5, 1, 3, 2, 4).reshape(1, c, 5 * s, 6 * s)
        torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_patch_layout_matches_torch(small):
    cfg, sd = small
    _, t = parse(pack.pack_bytes(sd, cfg, 98, 98))
    img = torch.randn(1, 3, 28, 42)
    w = torch.from_numpy(sd["pretrained.patch_embed.proj.weight"]).half().float()
    ref = F.conv2d(img, w, stride=14).flatten(2).transpose(1, 2)[0]          # [6, 384]
    p = img.reshape(3, 2, 14, 3, 14).permute(1, 3, 0, 2, 4)                  # [py, px, c, ky, kx]
    rows = torch.zeros(2, 3, 3, 14, 16)
    rows[..., :14] = p
    got = rows.reshape(6, 672) @ torch.from_numpy(t["patch.w"][:384, :672].astype(np.float32)).T
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_missing_key_and_bad_size_raise(small):
    cfg, sd = small
    bad = dict(sd)
    bad.pop("depth_head.scratch.output_conv1.weight")
    with pytest.raises(KeyError):
        pack.pack_bytes(bad, cfg, 98, 98)
    with pytest.raises(ValueError):
        pack.pack_bytes(sd, cfg, 100, 98)


def test_module_prefix_accepted(small):
    cfg, sd = small
    a = pack.pack_bytes({"module." + k: v for k, v in sd.items()}, cfg, 70, 70)
    b = pack.pack_bytes(sd, cfg, 70, 70)
    assert a == b
    assert pack.fingerprint(a) == pack.fingerprint(b) != pack.fingerprint(pack.pack_bytes(sd, cfg, 84, 84))


def test_layernorm_fold(small):
    """precision "fp16" packs fold norm1 / norm2 into qkv / fc1: LN(x) W^T + b
    == rstd * (x Wg^T - mean * c1) + c2 with the packed Wg (f16), c1, c2 and
    the row statistics from the 32-column (sum, sum of squares) partials --
    the arithmetic of the folded GEMM (gemm.hip), in float64 here."""
    cfg, sd = small
    o = pack.packed_tensors(sd, cfg, 98, 98, fold_ln=True)
    D = cfg["embed_dim"]
    x = torch.from_numpy(np.random.default_rng(0).standard_normal((5, D)).astype(np.float32) * 3 + 1)
    x = x.half().double()
    for blk, ln, lin, n in ((0, "norm1", "qkv", 3 * D), (3, "norm2", "fc1", cfg["mlp_hidden"])):
        p = f"pretrained.blocks.{blk}."
        w = sd[p + ("attn.qkv" if lin == "qkv" else "mlp.fc1") + ".weight"]
        b = sd[p + ("attn.qkv" if lin == "qkv" else "mlp.fc1") + ".bias"]
        g, bt = sd[p + ln + ".weight"], sd[p + ln + ".bias"]
        ref = F.layer_norm(x, (D,), torch.from_numpy(g).double(), torch.from_numpy(bt).double(), cfg["ln_eps"])
        ref = ref @ torch.from_numpy(w).half().double().T + torch.from_numpy(b).double()
        wg = torch.from_numpy(o[f"b{blk}.{lin}.wf"][:n, :D].astype(np.float64))
        c1 = torch.from_numpy(o[f"b{blk}.{lin}.c1"]).double()
        c2 = torch.from_numpy(o[f"b{blk}.{lin}.c2"]).double()
        part = x.reshape(5, D // 32, 32)
        mean = part.sum(-1).sum(-1) / D
        # Chan et al.'s merge of the slices' (sum, M2), as the GEMM prologue
        ms = part.mean(-1)
        m2 = ((part - ms[..., None]) ** 2).sum(-1) + 32 * (ms - mean[:, None]) ** 2
        rstd = 1.0 / torch.sqrt(m2.sum(-1) / D + cfg["ln_eps"])
        got = rstd[:, None] * (x @ wg.T - mean[:, None] * c1[None, :]) + c2[None, :]
        # f16 rounding of W * gamma vs of W (relative 2^-11 per weight)
        assert torch.allclose(got, ref, rtol=2e-3, atol=2e-3 * float(ref.abs().max())), (lin, (got - ref).abs().max())
    # the cls row's partials
    cls = torch.from_numpy(o["pos.cls"]).half().double().reshape(D // 32, 32)
    st = torch.from_numpy(o["pos.cls.st"]).double().reshape(D // 32, 2)
    assert torch.allclose(st[:, 0], cls.sum(-1), rtol=1e-6, atol=1e-5)
    assert torch.allclose(st[:, 1], ((cls - cls.mean(-1, keepdim=True)) ** 2).sum(-1), rtol=1e-6, atol=1e-5)
    # fp32-precision packs keep the unfolded layout only
    assert "b0.qkv.wf" not in pack.packed_tensors(sd, cfg, 98, 98)



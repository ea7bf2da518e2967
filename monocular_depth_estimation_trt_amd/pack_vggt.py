"""AOT weight packer for VGGT's depth path: upstream-keyed state dict ->
packed engine (family 2).

Replaces the reference's `models/vggt/onnx_export.py:78-131` (ONNX export of
`VGGTDepthOnlyWrapper` at 518x518 under fp16 autocast, with the export
patches of `core/export_compat.py`) and the TensorRT build of
`models/vggt/onnx2trt.py` for this model.  Same container as pack.py
(csrc/pack_format.h); what is folded at pack time:

* the aggregator's ImageNet normalisation into the patch-embed weights
  (W' = W / std_c, b' = b - sum W mean_c / std_c: the 14x14 stride-14 conv
  has no padding, so the fold is exact) -- the engine reads the [0, 1] images;
* cls + pos[0] and the 4 DINOv2 register tokens -> "pre.dino" [5][D]; the
  aggregator's camera + register tokens -> "pre.agg" [2][5][D] (set 0 =
  first frame of each batch item, set 1 = the others);
* the 2D RoPE tables cos/sin [max(gh, gw) + 2][16] (base 100, 32 features
  per axis, upstream _compute_frequency_components in fp32);
* the DPT head's UV sin/cos embeddings (ratio 0.1): after each 1x1
  projection as an f16 [np][oc_i] table the projection epilogue adds, and
  -- because output_conv2's first 3x3 conv is linear and zero-padded --
  the full-resolution one as conv(pe) without bias, an f16 [H*W][32] table
  the head epilogue adds before its ReLU (exact in real arithmetic,
  computed in float64);
* output_conv2's last 1x1 conv reduced to its depth channel (channel 1 is
  the confidence the wrapper drops, onnx_export.py:49-52).

A packed file is specific to one input size and one frame count S (the
global-attention length S * 1374 at 518^2), as the reference's engine is to
its static [1, S, 3, 518, 518] profile.
"""

from __future__ import annotations

import struct
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

from . import pack as PK
from . import weights_vggt as WV

FAMILY_VGGT = 2
NPRE = 1 + WV.NUM_REG      # camera + 4 register tokens ahead of the patch tokens


# ---- tables -----------------------------------------------------------------
def uv_grid(width: int, height: int, aspect: float) -> np.ndarray:
    """upstream heads/utils.create_uv_grid -> [height*width, 2] (u, v), float64."""
    diag = (aspect ** 2 + 1.0) ** 0.5
    sx, sy = aspect / diag, 1.0 / diag
    xs = np.linspace(-sx * (width - 1) / width, sx * (width - 1) / width, width)
    ys = np.linspace(-sy * (height - 1) / height, sy * (height - 1) / height, height)
    uu, vv = np.meshgrid(xs, ys, indexing="xy")
    return np.stack([uu.reshape(-1), vv.reshape(-1)], -1)


def _sincos(dim: int, pos: np.ndarray, omega_0: float) -> np.ndarray:
    omega = np.arange(dim // 2, dtype=np.float64) / (dim / 2.0)
    omega = 1.0 / omega_0 ** omega
    out = pos[:, None] * omega[None, :]
    return np.concatenate([np.sin(out), np.cos(out)], 1)


def uv_embed(channels: int, h: int, w: int, aspect: float, ratio: float = 0.1, omega_0: float = 100.0) -> np.ndarray:
    """ratio * position_grid_to_embed(create_uv_grid(w, h, aspect), C) -> [h*w, C] float64
    (token-major: row = y*w + x)."""
    g = uv_grid(w, h, aspect)
    return ratio * np.concatenate([_sincos(channels // 2, g[:, 0], omega_0),
                                   _sincos(channels // 2, g[:, 1], omega_0)], 1)


def rope_tables(npos: int, dim: int = 32, base: float = 100.0) -> Tuple[np.ndarray, np.ndarray]:
    """cos/sin [npos][dim/2] fp32: angle(p, j) = p * base^-(2j/dim), the
    non-duplicated half of upstream _compute_frequency_components (fp32)."""
    exps = (np.arange(0, dim, 2, dtype=np.float32) / np.float32(dim)).astype(np.float32)
    inv = (np.float32(1.0) / (np.float32(base) ** exps)).astype(np.float32)
    ang = (np.arange(npos, dtype=np.float32)[:, None] * inv[None, :]).astype(np.float32)
    return np.cos(ang).astype(np.float32), np.sin(ang).astype(np.float32)


def fold_patch_embed(w: np.ndarray, b: np.ndarray, mean=WV.RESNET_MEAN, std=WV.RESNET_STD):
    """Patch-embed conv over (x - mean) / std == conv with W' = W / std, b' =
    b - sum W mean / std (float64, returned float32)."""
    w64 = w.astype(np.float64)
    m = np.asarray(mean, np.float64)[None, :, None, None]
    s = np.asarray(std, np.float64)[None, :, None, None]
    wf = w64 / s
    bf = b.astype(np.float64) - (w64 * m / s).sum(axis=(1, 2, 3))
    return wf.astype(np.float32), bf.astype(np.float32)


def head_pe(w_conv: np.ndarray, h: int, w: int, ratio: float = 0.1, omega_0: float = 100.0) -> np.ndarray:
    """conv3x3(pad 1, no bias) of the full-resolution embedding through
    output_conv2.0 -> [h*w, Cout] float64."""
    import torch
    import torch.nn.functional as F
    cin = w_conv.shape[1]
    pe = uv_embed(cin, h, w, float(w) / float(h), ratio, omega_0).T.reshape(1, cin, h, w)
    with torch.no_grad():
        y = F.conv2d(torch.from_numpy(np.ascontiguousarray(pe)), torch.from_numpy(w_conv.astype(np.float64)),
                     padding=1)
    return y[0].reshape(w_conv.shape[0], h * w).T.numpy()


# ---- packing ----------------------------------------------------------------
def _blk(o, sd, src: str, dst: str, qk_norm: bool):
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1)  # noqa: E731
    o[dst + "ln1.g"] = f32(sd[src + "norm1.weight"])
    o[dst + "ln1.b"] = f32(sd[src + "norm1.bias"])
    o[dst + "qkv.w"] = PK._pad2(sd[src + "attn.qkv.weight"])
    o[dst + "qkv.b"] = f32(sd[src + "attn.qkv.bias"])
    if qk_norm:
        o[dst + "qn.g"] = f32(sd[src + "attn.q_norm.weight"])
        o[dst + "qn.b"] = f32(sd[src + "attn.q_norm.bias"])
        o[dst + "kn.g"] = f32(sd[src + "attn.k_norm.weight"])
        o[dst + "kn.b"] = f32(sd[src + "attn.k_norm.bias"])
    o[dst + "proj.w"] = PK._pad2(sd[src + "attn.proj.weight"])
    o[dst + "proj.b"] = f32(sd[src + "attn.proj.bias"])
    o[dst + "ls1"] = f32(sd[src + "ls1.gamma"])
    o[dst + "ln2.g"] = f32(sd[src + "norm2.weight"])
    o[dst + "ln2.b"] = f32(sd[src + "norm2.bias"])
    o[dst + "fc1.w"] = PK._pad2(sd[src + "mlp.fc1.weight"])
    o[dst + "fc1.b"] = f32(sd[src + "mlp.fc1.bias"])
    o[dst + "fc2.w"] = PK._pad2(sd[src + "mlp.fc2.weight"])
    o[dst + "fc2.b"] = f32(sd[src + "mlp.fc2.bias"])
    o[dst + "ls2"] = f32(sd[src + "ls2.gamma"])


def packed_tensors(sd: Dict[str, np.ndarray], cfg: dict) -> "OrderedDict[str, np.ndarray]":
    sd = PK.normalize_keys(sd)
    missing = [k for k in WV.expected_keys(cfg) if k not in sd and not k.endswith("mask_token")]
    if missing:
        raise KeyError(f"VGGT state dict lacks {len(missing)} keys, e.g. {missing[:4]}")
    D, P, S = cfg["embed_dim"], cfg["patch"], cfg["img"]
    g = S // P
    np_ = g * g
    oc = cfg["out_channels"]
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1)  # noqa: E731
    o: "OrderedDict[str, np.ndarray]" = OrderedDict()
    p = "aggregator.patch_embed."
    pw, pb = fold_patch_embed(sd[p + "patch_embed.proj.weight"], sd[p + "patch_embed.proj.bias"])
    pe16 = np.zeros((D, 3, P, 16), np.float32)
    pe16[..., :P] = pw
    o["patch.w"] = PK._pad2(pe16.reshape(D, 3 * P * 16))
    o["patch.b"] = f32(pb)
    pos = sd[p + "pos_embed"]
    if pos.shape[1] != 1 + np_:
        raise ValueError(f"pos_embed holds {pos.shape[1] - 1} positions; the packed size {S} needs {np_} "
                         "(pack at the checkpoint's 518x518 grid)")
    o["pos.patch"] = np.ascontiguousarray(pos[0, 1:], dtype=np.float32)
    o["pre.dino"] = np.ascontiguousarray(np.concatenate(
        [sd[p + "cls_token"].reshape(1, D) + pos[0, :1], sd[p + "register_tokens"].reshape(WV.NUM_REG, D)], 0),
        dtype=np.float32)
    for i in range(cfg["depth"]):
        _blk(o, sd, f"{p}blocks.{i}.", f"db{i}.", False)
    o["norm.g"] = f32(sd[p + "norm.weight"])
    o["norm.b"] = f32(sd[p + "norm.bias"])
    a = "aggregator."
    cam = sd[a + "camera_token"].reshape(2, 1, D)
    reg = sd[a + "register_token"].reshape(2, WV.NUM_REG, D)
    o["pre.agg"] = np.ascontiguousarray(np.concatenate([cam, reg], 1), dtype=np.float32)   # [2][5][D]
    for i in range(cfg["aa_depth"]):
        _blk(o, sd, f"{a}frame_blocks.{i}.", f"fb{i}.", True)
        _blk(o, sd, f"{a}global_blocks.{i}.", f"gb{i}.", True)
    cos, sin = rope_tables(g + 2, 32, cfg["rope_freq"])
    o["rope.cos"] = cos
    o["rope.sin"] = sin
    h = "depth_head."
    o["dh.norm.g"] = f32(sd[h + "norm.weight"])
    o["dh.norm.b"] = f32(sd[h + "norm.bias"])
    for i in range(4):
        w = sd[f"{h}projects.{i}.weight"]
        o[f"proj{i}.w"] = PK._pad2(w.reshape(w.shape[0], w.shape[1]))
        o[f"proj{i}.b"] = f32(sd[f"{h}projects.{i}.bias"])
        o[f"pe{i}"] = uv_embed(oc[i], g, g, 1.0, cfg["pe_ratio"], cfg["pe_omega"]).astype(np.float16)
    o["rs0.w"] = PK._convT(sd[h + "resize_layers.0.weight"])
    o["rs0.b"] = f32(sd[h + "resize_layers.0.bias"])
    o["rs1.w"] = PK._convT(sd[h + "resize_layers.1.weight"])
    o["rs1.b"] = f32(sd[h + "resize_layers.1.bias"])
    o["rs3.w"] = PK._conv3(sd[h + "resize_layers.3.weight"])
    o["rs3.b"] = f32(sd[h + "resize_layers.3.bias"])
    for i in range(4):
        o[f"rn{i + 1}.w"] = PK._conv3(sd[f"{h}scratch.layer{i + 1}_rn.weight"], -(-oc[i] // 32) * 32)
    for r in range(1, 5):
        s = f"{h}scratch.refinenet{r}."
        w = sd[s + "out_conv.weight"]
        o[f"rf{r}.out.w"] = PK._pad2(w.reshape(w.shape[0], w.shape[1]))
        o[f"rf{r}.out.b"] = f32(sd[s + "out_conv.bias"])
        for u in ((2,) if r == 4 else (1, 2)):
            for c in (1, 2):
                o[f"rf{r}.rcu{u}.c{c}.w"] = PK._conv3(sd[f"{s}resConfUnit{u}.conv{c}.weight"])
                o[f"rf{r}.rcu{u}.c{c}.b"] = f32(sd[f"{s}resConfUnit{u}.conv{c}.bias"])
    s = h + "scratch."
    o["head.c1.w"] = PK._conv3(sd[s + "output_conv1.weight"])
    o["head.c1.b"] = f32(sd[s + "output_conv1.bias"])
    w2 = sd[s + "output_conv2.0.weight"]
    o["head.c2.w"] = PK._conv3(w2)
    o["head.c2.b"] = f32(sd[s + "output_conv2.0.bias"])
    o["head.pe"] = head_pe(w2, S, S, cfg["pe_ratio"], cfg["pe_omega"]).astype(np.float16)
    o["head.c3.w"] = f32(sd[s + "output_conv2.2.weight"][0])          # depth channel only
    o["head.c3.b"] = f32(sd[s + "output_conv2.2.bias"][:1])
    return o


def config_bytes(cfg: dict, frames: int) -> bytes:
    """PackConfig (csrc/pack_format.h) with family = 2: the DA-V2 fields carry
    the DINOv2 geometry (depth = DINOv2 blocks, ln_eps its eps, metric = 2:
    exp head), then the family block (zeros but family) and the VGGT fields
    (frames, special tokens, aggregator depth, aggregator LayerNorm eps)."""
    if frames < 1:
        raise ValueError(f"frames must be >= 1, got {frames}")
    S = cfg["img"]
    b = struct.pack("<8i4i4i2i2f16s", cfg["embed_dim"], cfg["depth"], cfg["num_heads"], cfg["mlp_hidden"],
                    cfg["patch"], S, S, cfg["features"], *cfg["out_channels"], *cfg["taps"], cfg["head_hidden"], 2,
                    0.0, float(cfg["ln_eps"]), cfg["encoder"].encode()[:15])
    b += struct.pack("<if3f3f", 0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    assert len(b) == 128, len(b)
    b += struct.pack("<6i2i2i3i", FAMILY_VGGT, *([0] * 12))
    assert len(b) == 180, len(b)
    b += struct.pack("<3if", int(frames), NPRE, cfg["aa_depth"], float(cfg["agg_eps"]))
    assert len(b) == 196, len(b)
    return b + b"\0" * 60


def pack_bytes(sd: Dict[str, np.ndarray], cfg: dict, frames: int = 1) -> bytes:
    return PK.container(packed_tensors(sd, cfg), config_bytes(cfg, frames))


def synthetic_blob(preset: str = "vggt_1b", frames: int = 1, seed: int = 2468):
    cfg = WV.vggt_config(preset)
    return pack_bytes(WV.synthetic_state_dict(cfg, seed), cfg, frames), cfg

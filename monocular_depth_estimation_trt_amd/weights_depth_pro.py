"""Depth Pro model configuration and the seeded synthetic checkpoint.

The reference builds Depth Pro from apple/ml-depth-pro with
`DepthProConfig(patch_encoder_preset="dinov2l16_384",
image_encoder_preset="dinov2l16_384", decoder_features=256,
use_fov_head=True, fov_encoder_preset="dinov2l16_384")`
(`models/depth_pro/onnx_export.py:13-22`) and exports it at its fixed
1536x1536 input (`models/depth_pro/spec.json`, `onnx2trt.py:45`).  That
upstream repository is not vendored and its checkpoint is not reachable
offline, so -- as for Depth Anything V2 -- every parity test and benchmark runs
on synthetic weights drawn here.

Key names are transformers' `DepthProForDepthEstimation` names (the
`apple/DepthPro-hf` checkpoint layout; HF:models/depth_pro/modeling_depth_pro.py),
which the in-container oracle cross-check loads directly.  The ViT geometry
(three DINOv2-L/16 encoders at 384x384 -> 24x24 tokens + cls) and the decoder
widths follow HF's DepthProConfig defaults, which restate the upstream preset:
hooks [11, 5], scaled-image feature dims [1024, 1024, 512], intermediate dims
[256, 256], fusion 256, 2 FOV head layers, merge padding 3.

Scales: as weights.py -- W ~ N(0, 1/fan_in), LayerScale ~0.5,
LayerNorm gamma 1 +- 0.1, biases N(0, 0.02^2), cls/pos N(0, 0.5^2); the depth
head's last bias is drawn around +0.5 so the final ReLU leaves most of the map
positive (a map that is mostly 0 is a weak parity signal).
"""

from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

LN_EPS = 1e-6
HEAD_HIDDEN = 32   # HF DepthProDepthEstimationHead: Conv2d(features // 2, 32, 3)

# encoder presets (one DINOv2 geometry shared by patch / image / fov encoders)
VIT = {
    "dinov2l16_384": dict(embed_dim=1024, depth=24, num_heads=16),
    # reduced widths with the same 384/16 token geometry: parity fixtures
    "tiny": dict(embed_dim=128, depth=4, num_heads=2),
    # the real widths (D 1024, 16 heads, decoder 256, scaled dims 1024/1024/512)
    # with 4 instead of 24 blocks per encoder: the full-width parity fixture
    "dinov2l16_384_shallow": dict(embed_dim=1024, depth=4, num_heads=16),
}


def depth_pro_config(preset: str = "dinov2l16_384", use_fov: bool = True, **over) -> dict:
    """Architecture constants.  `preset="tiny"` keeps every shape rule of the
    1536x1536 model (35 patches of 384^2, 24x24 tokens, identity merges)
    with narrow layers, so the CPU oracle finishes in seconds."""
    if preset not in VIT:
        raise ValueError(f"unknown Depth Pro preset {preset!r}; have {sorted(VIT)}")
    cfg = dict(VIT[preset])
    if preset == "tiny":
        cfg.update(hooks=[3, 1], inter_dims=[128, 128], scaled_dims=[256, 256, 128], fusion=128)
    elif preset == "dinov2l16_384_shallow":
        cfg.update(hooks=[3, 1], inter_dims=[256, 256], scaled_dims=[1024, 1024, 512], fusion=256)
    else:
        cfg.update(hooks=[11, 5], inter_dims=[256, 256], scaled_dims=[1024, 1024, 512], fusion=256)
    cfg.update(family="depth_pro", encoder=preset, patch=16, vit_size=384, img=1536,
               mlp_hidden=4 * cfg["embed_dim"], ratios=[0.25, 0.5, 1.0], overlaps=[0.0, 0.5, 0.25],
               merge_pad=3, head_hidden=HEAD_HIDDEN, use_fov=bool(use_fov), fov_layers=2, ln_eps=LN_EPS)
    cfg.update(over)
    return cfg


def _vit_spec(pfx: str, cfg: dict) -> List[Tuple[str, Tuple[int, ...], str, float]]:
    D, P = cfg["embed_dim"], cfg["patch"]
    G = cfg["vit_size"] // P
    e = pfx + "embeddings."
    s = [(e + "cls_token", (1, 1, D), "tok", 0), (e + "mask_token", (1, D), "zero", 0),
         (e + "position_embeddings", (1, 1 + G * G, D), "tok", 0),
         (e + "patch_embeddings.projection.weight", (D, 3, P, P), "w", 3 * P * P),
         (e + "patch_embeddings.projection.bias", (D,), "b", 0)]
    for i in range(cfg["depth"]):
        b = f"{pfx}encoder.layer.{i}."
        s += [(b + "norm1.weight", (D,), "g", 0), (b + "norm1.bias", (D,), "b", 0)]
        for n in ("query", "key", "value"):
            s += [(f"{b}attention.attention.{n}.weight", (D, D), "w", D),
                  (f"{b}attention.attention.{n}.bias", (D,), "b", 0)]
        s += [(b + "attention.output.dense.weight", (D, D), "w", D),
              (b + "attention.output.dense.bias", (D,), "b", 0),
              (b + "layer_scale1.lambda1", (D,), "ls", 0),
              (b + "norm2.weight", (D,), "g", 0), (b + "norm2.bias", (D,), "b", 0),
              (b + "mlp.fc1.weight", (4 * D, D), "w", D), (b + "mlp.fc1.bias", (4 * D,), "b", 0),
              (b + "mlp.fc2.weight", (D, 4 * D), "w", 4 * D), (b + "mlp.fc2.bias", (D,), "b", 0),
              (b + "layer_scale2.lambda1", (D,), "ls", 0)]
    s += [(pfx + "layernorm.weight", (D,), "g", 0), (pfx + "layernorm.bias", (D,), "b", 0)]
    return s


def _rcu_spec(pfx: str, F: int):
    s = []
    for u in (1, 2):
        for c in (1, 2):
            s += [(f"{pfx}residual_layer{u}.convolution{c}.weight", (F, F, 3, 3), "w", 9 * F),
                  (f"{pfx}residual_layer{u}.convolution{c}.bias", (F,), "b", 0)]
    return s


def _spec(cfg: dict) -> List[Tuple[str, Tuple[int, ...], str, float]]:
    """(key, shape, kind, fan_in) in the fixed draw order of the RNG."""
    D, F = cfg["embed_dim"], cfg["fusion"]
    sd_, idims = cfg["scaled_dims"], cfg["inter_dims"]
    s = []
    s += _vit_spec("depth_pro.encoder.patch_encoder.model.", cfg)
    s += _vit_spec("depth_pro.encoder.image_encoder.model.", cfg)
    u = "depth_pro.neck.feature_upsample."
    s += [(u + "image_block.layers.0.weight", (D, sd_[0], 2, 2), "w", D),
          (u + "image_block.layers.0.bias", (sd_[0],), "b", 0)]
    for i, fd in enumerate(sd_):
        s += [(f"{u}scaled_images.{i}.layers.0.weight", (fd, D, 1, 1), "w", D),
              (f"{u}scaled_images.{i}.layers.1.weight", (fd, fd, 2, 2), "w", fd)]
    for i, fd in enumerate(idims):
        mid = F if i == 0 else fd
        s += [(f"{u}intermediate.{i}.layers.0.weight", (mid, D, 1, 1), "w", D)]
        for j in range(2 + i):
            cin = mid if j == 0 else fd
            s += [(f"{u}intermediate.{i}.layers.{j + 1}.weight", (cin, fd, 2, 2), "w", cin)]
    n = "depth_pro.neck."
    s += [(n + "fuse_image_with_low_res.weight", (sd_[0], 2 * sd_[0], 1, 1), "w", 2 * sd_[0]),
          (n + "fuse_image_with_low_res.bias", (sd_[0],), "b", 0)]
    comb = list(sd_) + list(idims)
    for i, cin in enumerate(comb):
        if i == len(comb) - 1 and cin == F:
            continue  # nn.Identity
        s += [(f"{n}feature_projection.projections.{i}.weight", (F, cin, 3, 3), "w", 9 * cin)]
    nl = len(cfg["hooks"]) + len(cfg["ratios"])
    for i in range(nl - 1):
        f = f"fusion_stage.intermediate.{i}."
        s += _rcu_spec(f, F)
        s += [(f + "deconv.weight", (F, F, 2, 2), "w", F),
              (f + "projection.weight", (F, F, 1, 1), "w", F), (f + "projection.bias", (F,), "b", 0)]
    f = "fusion_stage.final."
    s += _rcu_spec(f, F)
    s += [(f + "projection.weight", (F, F, 1, 1), "w", F), (f + "projection.bias", (F,), "b", 0)]
    H2 = cfg["head_hidden"]
    s += [("head.layers.0.weight", (F // 2, F, 3, 3), "w", 9 * F), ("head.layers.0.bias", (F // 2,), "b", 0),
          ("head.layers.1.weight", (F // 2, F // 2, 2, 2), "w", F // 2), ("head.layers.1.bias", (F // 2,), "b", 0),
          ("head.layers.2.weight", (H2, F // 2, 3, 3), "w", 9 * (F // 2)), ("head.layers.2.bias", (H2,), "b", 0),
          ("head.layers.4.weight", (1, H2, 1, 1), "w", H2), ("head.layers.4.bias", (1,), "bpos", 0)]
    if cfg["use_fov"]:
        fv = "fov_model."
        s += _vit_spec(fv + "fov_encoder.model.", cfg)
        s += [(fv + "fov_encoder.neck.weight", (F // 2, D), "w", D), (fv + "fov_encoder.neck.bias", (F // 2,), "b", 0),
              (fv + "conv.weight", (F // 2, F, 3, 3), "w", 9 * F), (fv + "conv.bias", (F // 2,), "b", 0)]
        c = F // 2
        for i in range(cfg["fov_layers"]):
            s += [(f"{fv}head.layers.{2 * i}.weight", (c // 2, c, 3, 3), "w", 9 * c),
                  (f"{fv}head.layers.{2 * i}.bias", (c // 2,), "b", 0)]
            c //= 2
        k = fov_final_kernel(cfg)
        s += [(f"{fv}head.layers.{2 * cfg['fov_layers']}.weight", (1, c, k, k), "w", c * k * k),
              (f"{fv}head.layers.{2 * cfg['fov_layers']}.bias", (1,), "b", 0)]
    return s


def fov_final_kernel(cfg: dict) -> int:
    """HF DepthProFovHead final conv size: int((out_size - 1) / 2**layers + 1)."""
    out = cfg["vit_size"] // cfg["patch"]
    return int((out - 1) / 2 ** cfg["fov_layers"] + 1)


def synthetic_state_dict(cfg: dict, seed: int = 4321) -> "OrderedDict[str, np.ndarray]":
    rng = np.random.Generator(np.random.PCG64(seed))
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape, kind, fan_in in _spec(cfg):
        if kind == "zero":
            a = np.zeros(shape, np.float32)
        else:
            z = rng.standard_normal(shape, dtype=np.float32)
            if kind == "w":
                a = z * np.float32(1.0 / np.sqrt(fan_in))
            elif kind == "b":
                a = z * np.float32(0.02)
            elif kind == "bpos":
                a = np.float32(0.5) + z * np.float32(0.02)
            elif kind == "g":
                a = np.float32(1.0) + z * np.float32(0.1)
            elif kind == "ls":
                a = np.float32(0.5) + z * np.float32(0.05)
            elif kind == "tok":
                a = z * np.float32(0.5)
            else:  # pragma: no cover
                raise AssertionError(kind)
        out[key] = np.ascontiguousarray(a, dtype=np.float32)
    return out


def expected_keys(cfg: dict) -> List[str]:
    return [k for k, *_ in _spec(cfg)]


def expected_shapes(cfg: dict) -> Dict[str, Tuple[int, ...]]:
    return {k: tuple(s) for k, s, *_ in _spec(cfg)}


def state_dict_digest(sd: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        a = np.ascontiguousarray(np.asarray(sd[k], dtype=np.float32))
        h.update(k.encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def synthetic_images(batch: int, size: int = 1536, first_seed: int = 0) -> np.ndarray:
    """The Depth Pro input domain: u ~ U{0..255} (PCG64 seed i for image i),
    then (u/255 - 0.5)/0.5 (`models/depth_pro/onnx2trt.py:66-70`,
    Normalize([0.5]*3, [0.5]*3)) -> float32 NCHW [batch, 3, size, size]."""
    out = np.empty((batch, 3, size, size), np.float32)
    for i in range(batch):
        rng = np.random.Generator(np.random.PCG64(first_seed + i))
        u = rng.integers(0, 256, size=(size, size, 3), dtype=np.uint8)
        out[i] = ((u.astype(np.float32) / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)).transpose(2, 0, 1)
    return out

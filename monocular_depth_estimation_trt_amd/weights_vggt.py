"""VGGT model configuration and the seeded synthetic checkpoint.

The reference exports facebookresearch/vggt's `VGGT` wrapped as
`VGGTDepthOnlyWrapper` (`models/vggt/onnx_export.py:38-52`): the aggregator
plus the depth head only, input "images" [1, S=1, 3, 518, 518] in [0, 1]
(`models/vggt/spec.json`: /255, no mean/std -- the aggregator normalises with
the ImageNet statistics itself), output "depth" [1, 1, 518, 518, 1].  The
checkpoint is `facebook/VGGT-1B/model.pt` (`onnx_export.py:55-75`), not
reachable offline, and the upstream repository is not vendored, so every
parity test and benchmark runs on synthetic weights drawn here with the
upstream key names (a real `model.pt` on a box that has one packs unchanged;
the camera / point / track heads' keys are ignored).

Architecture (upstream VGGT-1B, restated; the reference's TensorRT profile
`reports/profile/vggt.json` confirms the module tree: aggregator/patch_embed/
blocks.0-23, aggregator/frame_blocks.0-23, aggregator/global_blocks.0-23,
depth_head/{projects,resize_layers,layerN_rn,refinenetN,output_conv1,
output_conv2}; `models/vggt/onnx_export_split.py:49-59` gives the token
layout: 24 x [B, S, 1374, 2048], patch_start_idx 5):

* patch_embed = DINOv2 ViT-L/14 with 4 register tokens (img_size 518,
  LayerScale, LN eps 1e-6), its final norm's patch tokens are the frame tokens;
* 5 special tokens per frame (1 camera + 4 register; frame 0 of each batch
  item uses set 0, the others set 1);
* 24 x (frame-attention block, global-attention block): pre-LN (eps 1e-5)
  blocks with per-head q/k LayerNorm and 2D RoPE (frequency 100) on the
  patch-grid positions (+1; special tokens at (0, 0)), LayerScale, GELU MLP;
* depth head = DPT on cat(frame_out[i], global_out[i]) for i in [4,11,17,23]
  (2048 channels, LayerNorm eps 1e-5), features 256, out_channels
  [256,512,1024,1024], UV sin/cos positional embeddings (ratio 0.1) after the
  projections and after the final upsample, in-place-ReLU residual units,
  output_conv2 -> 2 channels, depth = exp(channel 0).

Scales: as weights.py: W ~ N(0, 1/fan_in), LayerScale ~0.5,
LayerNorm gamma 1 +- 0.1, biases N(0, 0.02^2), tokens N(0, 0.5^2).
"""

from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

PATCH = 14
NUM_REG = 4            # DINOv2 register tokens == aggregator register tokens
DINO_EPS = 1e-6        # DINOv2 LayerNorm
AGG_EPS = 1e-5         # nn.LayerNorm default: aggregator blocks, q/k norm, depth-head norm
HEAD_HIDDEN = 32       # DPTHead head_features_2
RESNET_MEAN = (0.485, 0.456, 0.406)
RESNET_STD = (0.229, 0.224, 0.225)

PRESETS = {
    # VGGT-1B: DINOv2-L/14-reg patch embed + 24 frame/global block pairs
    "vggt_1b": dict(embed_dim=1024, num_heads=16, depth=24, aa_depth=24, features=256,
                    out_channels=[256, 512, 1024, 1024], taps=[4, 11, 17, 23], img=518),
    # the full widths and the 518^2 geometry with 2 + 4 blocks: every kernel
    # shape of VGGT-1B at a twelfth of its depth (GPU parity at full size)
    "vggt_1b_shallow": dict(embed_dim=1024, num_heads=16, depth=2, aa_depth=4, features=256,
                            out_channels=[256, 512, 1024, 1024], taps=[0, 1, 2, 3], img=518),
    # narrow layers and a 98x98 input (7x7 patches): CPU-fast parity fixtures
    "tiny": dict(embed_dim=128, num_heads=2, depth=2, aa_depth=4, features=64,
                 out_channels=[32, 64, 128, 128], taps=[0, 1, 2, 3], img=98),
}


def vggt_config(preset: str = "vggt_1b", **over) -> dict:
    if preset not in PRESETS:
        raise ValueError(f"unknown VGGT preset {preset!r}; have {sorted(PRESETS)}")
    cfg = dict(PRESETS[preset])
    cfg.update(family="vggt", encoder=preset, patch=PATCH, num_register=NUM_REG,
               mlp_hidden=4 * cfg["embed_dim"], head_hidden=HEAD_HIDDEN, ln_eps=DINO_EPS,
               agg_eps=AGG_EPS, rope_freq=100.0, pe_ratio=0.1, pe_omega=100.0, out_dim=2)
    cfg.update(over)
    if cfg["img"] % PATCH:
        raise ValueError(f"image size {cfg['img']} is not a multiple of {PATCH}")
    if sorted(cfg["taps"]) != list(cfg["taps"]) or not all(0 <= t < cfg["aa_depth"] for t in cfg["taps"]):
        raise ValueError(f"taps {cfg['taps']} must be increasing block indices below {cfg['aa_depth']}")
    return cfg


def _block(s, b: str, D: int, qk_norm: bool):
    s += [(b + "norm1.weight", (D,), "g", 0), (b + "norm1.bias", (D,), "b", 0),
          (b + "attn.qkv.weight", (3 * D, D), "w", D), (b + "attn.qkv.bias", (3 * D,), "b", 0)]
    if qk_norm:
        s += [(b + "attn.q_norm.weight", (64,), "g", 0), (b + "attn.q_norm.bias", (64,), "b", 0),
              (b + "attn.k_norm.weight", (64,), "g", 0), (b + "attn.k_norm.bias", (64,), "b", 0)]
    s += [(b + "attn.proj.weight", (D, D), "w", D), (b + "attn.proj.bias", (D,), "b", 0),
          (b + "ls1.gamma", (D,), "ls", 0),
          (b + "norm2.weight", (D,), "g", 0), (b + "norm2.bias", (D,), "b", 0),
          (b + "mlp.fc1.weight", (4 * D, D), "w", D), (b + "mlp.fc1.bias", (4 * D,), "b", 0),
          (b + "mlp.fc2.weight", (D, 4 * D), "w", 4 * D), (b + "mlp.fc2.bias", (D,), "b", 0),
          (b + "ls2.gamma", (D,), "ls", 0)]


def _spec(cfg: dict) -> List[Tuple[str, Tuple[int, ...], str, float]]:
    """(key, shape, kind, fan_in) in a fixed order -- the draw order of the RNG."""
    D, F, P = cfg["embed_dim"], cfg["features"], cfg["patch"]
    oc = cfg["out_channels"]
    G = cfg["img"] // P
    s: List[Tuple[str, Tuple[int, ...], str, float]] = []
    p = "aggregator.patch_embed."
    s += [(p + "cls_token", (1, 1, D), "tok", 0), (p + "pos_embed", (1, 1 + G * G, D), "tok", 0),
          (p + "register_tokens", (1, NUM_REG, D), "tok", 0), (p + "mask_token", (1, D), "zero", 0),
          (p + "patch_embed.proj.weight", (D, 3, P, P), "w", 3 * P * P),
          (p + "patch_embed.proj.bias", (D,), "b", 0)]
    for i in range(cfg["depth"]):
        _block(s, f"{p}blocks.{i}.", D, False)
    s += [(p + "norm.weight", (D,), "g", 0), (p + "norm.bias", (D,), "b", 0)]
    a = "aggregator."
    s += [(a + "camera_token", (1, 2, 1, D), "tok", 0), (a + "register_token", (1, 2, NUM_REG, D), "tok", 0)]
    for i in range(cfg["aa_depth"]):
        _block(s, f"{a}frame_blocks.{i}.", D, True)
    for i in range(cfg["aa_depth"]):
        _block(s, f"{a}global_blocks.{i}.", D, True)
    h = "depth_head."
    C2 = 2 * D
    s += [(h + "norm.weight", (C2,), "g", 0), (h + "norm.bias", (C2,), "b", 0)]
    for i in range(4):
        s += [(f"{h}projects.{i}.weight", (oc[i], C2, 1, 1), "w", C2),
              (f"{h}projects.{i}.bias", (oc[i],), "b", 0)]
    s += [(h + "resize_layers.0.weight", (oc[0], oc[0], 4, 4), "w", oc[0]),
          (h + "resize_layers.0.bias", (oc[0],), "b", 0),
          (h + "resize_layers.1.weight", (oc[1], oc[1], 2, 2), "w", oc[1]),
          (h + "resize_layers.1.bias", (oc[1],), "b", 0),
          (h + "resize_layers.3.weight", (oc[3], oc[3], 3, 3), "w", 9 * oc[3]),
          (h + "resize_layers.3.bias", (oc[3],), "b", 0)]
    for i in range(4):
        s += [(f"{h}scratch.layer{i + 1}_rn.weight", (F, oc[i], 3, 3), "w", 9 * oc[i])]
    for r in range(1, 5):
        rb = f"{h}scratch.refinenet{r}."
        s += [(rb + "out_conv.weight", (F, F, 1, 1), "w", F), (rb + "out_conv.bias", (F,), "b", 0)]
        for u in ((2,) if r == 4 else (1, 2)):   # refinenet4: has_residual=False
            for c in (1, 2):
                s += [(f"{rb}resConfUnit{u}.conv{c}.weight", (F, F, 3, 3), "w", 9 * F),
                      (f"{rb}resConfUnit{u}.conv{c}.bias", (F,), "b", 0)]
    H2 = cfg["head_hidden"]
    s += [(h + "scratch.output_conv1.weight", (F // 2, F, 3, 3), "w", 9 * F),
          (h + "scratch.output_conv1.bias", (F // 2,), "b", 0),
          (h + "scratch.output_conv2.0.weight", (H2, F // 2, 3, 3), "w", 9 * (F // 2)),
          (h + "scratch.output_conv2.0.bias", (H2,), "b", 0),
          (h + "scratch.output_conv2.2.weight", (cfg["out_dim"], H2, 1, 1), "w", H2),
          (h + "scratch.output_conv2.2.bias", (cfg["out_dim"],), "b", 0)]
    return s


def expected_keys(cfg: dict) -> List[str]:
    return [k for k, *_ in _spec(cfg)]


def expected_shapes(cfg: dict) -> Dict[str, Tuple[int, ...]]:
    return {k: shape for k, shape, *_ in _spec(cfg)}


def synthetic_state_dict(cfg: dict, seed: int = 2468) -> "OrderedDict[str, np.ndarray]":
    """Seeded, fan-in scaled upstream-keyed state dict (float32 numpy)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for key, shape, kind, fan_in in _spec(cfg):
        if kind == "zero":
            a = np.zeros(shape, np.float32)
        else:
            a = rng.standard_normal(shape, dtype=np.float32)
            if kind == "w":
                a *= np.float32(1.0 / np.sqrt(fan_in))
            elif kind == "b":
                a *= np.float32(0.02)
            elif kind == "g":
                a = np.float32(1.0) + a * np.float32(0.1)
            elif kind == "ls":
                a = np.float32(0.5) + a * np.float32(0.05)
            elif kind == "tok":
                a *= np.float32(0.5)
            else:  # pragma: no cover
                raise AssertionError(kind)
        out[key] = np.ascontiguousarray(a, dtype=np.float32)
    return out


def state_dict_digest(sd: Dict[str, np.ndarray]) -> str:
    """sha256 over keys + raw float32 bytes, in key order."""
    h = hashlib.sha256()
    for k in sorted(sd):
        a = np.ascontiguousarray(np.asarray(sd[k], dtype=np.float32))
        h.update(k.encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def synthetic_images(batch: int, frames: int, size: int, first_seed: int = 0) -> np.ndarray:
    """The reference's input domain: u ~ U{0..255} per pixel (PCG64 seed
    first_seed + index), /255 in float64 -> float32 [B, S, 3, H, W] in [0, 1]
    (`models/vggt/spec.json` normalize: scale 255, no mean/std)."""
    out = np.empty((batch, frames, 3, size, size), np.float32)
    flat = out.reshape(batch * frames, 3, size, size)
    for i in range(batch * frames):
        rng = np.random.Generator(np.random.PCG64(first_seed + i))
        u = rng.integers(0, 256, size=(size, size, 3), dtype=np.uint8)
        flat[i] = (u.astype(np.float64) / 255.0).transpose(2, 0, 1)
    return out

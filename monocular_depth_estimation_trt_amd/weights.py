"""Model configurations and the seeded synthetic checkpoint.

No Depth Anything V2 checkpoint is reachable offline (the reference downloads
them from HuggingFace, `models/depth_anything_v2/README.md:61-73`), so every
parity test and every benchmark runs on synthetic weights drawn here.  The
state dict uses the *upstream* key names -- the names
`torch.load(depth_anything_v2_metric_hypersim_vits.pth)` returns in
`models/depth_anything_v2/infer_metric.py:67-68` -- so the AOT packer
(`pack.py`) accepts a real checkpoint on a box that has one, unchanged.

Encoder table: `models/depth_anything_v2/infer.py:55-60` (features /
out_channels) and upstream `DepthAnythingV2.intermediate_layer_idx` (tap
blocks).  Metric head: `max_depth` 20 (hypersim) / 80 (vkitti),
`models/depth_anything_v2/infer_metric.py:61-66`.

Scales: W ~ N(0, 1/fan_in), LayerScale ~0.5,
LayerNorm gamma ~ 1 +- 0.1, biases N(0, 0.02^2), cls/pos tokens N(0, 0.5^2).
With HF's default init the output is flat (9.9992-10.0003) and useless as a
parity signal; these scales give a depth map that depends on the input.
"""

from __future__ import annotations

import hashlib
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

PATCH = 14
POS_GRID = 37          # upstream DINOv2 is built with img_size=518 -> 37x37 grid
HEAD_HIDDEN = 32       # upstream DPTHead head_features_2
LN_EPS = 1e-6

ENCODERS = {
    "vits": dict(embed_dim=384, depth=12, num_heads=6, features=64,
                 out_channels=[48, 96, 192, 384], taps=[2, 5, 8, 11]),
    "vitb": dict(embed_dim=768, depth=12, num_heads=12, features=128,
                 out_channels=[96, 192, 384, 768], taps=[2, 5, 8, 11]),
    "vitl": dict(embed_dim=1024, depth=24, num_heads=16, features=256,
                 out_channels=[256, 512, 1024, 1024], taps=[4, 11, 17, 23]),
}


def model_config(encoder: str = "vits", depth_type: str = "metric",
                 max_depth: float = 20.0) -> dict:
    """The architecture constants of one DA-V2 variant."""
    if encoder not in ENCODERS:
        raise ValueError(f"unknown encoder {encoder!r}; have {sorted(ENCODERS)}")
    if depth_type not in ("metric", "relative"):
        raise ValueError(f"depth_type must be 'metric' or 'relative', got {depth_type!r}")
    cfg = dict(ENCODERS[encoder])
    cfg.update(encoder=encoder, depth_type=depth_type,
               max_depth=float(max_depth if depth_type == "metric" else 1.0),
               patch=PATCH, pos_grid=POS_GRID, mlp_hidden=4 * cfg["embed_dim"],
               head_hidden=HEAD_HIDDEN, ln_eps=LN_EPS)
    return cfg


def _spec(cfg: dict) -> List[Tuple[str, Tuple[int, ...], str, float]]:
    """(key, shape, kind, fan_in) in a fixed order -- the draw order of the RNG."""
    D, F = cfg["embed_dim"], cfg["features"]
    oc = cfg["out_channels"]
    G = cfg["pos_grid"]
    s: List[Tuple[str, Tuple[int, ...], str, float]] = []
    p = "pretrained."
    s += [(p + "cls_token", (1, 1, D), "tok", 0), (p + "pos_embed", (1, 1 + G * G, D), "tok", 0),
          (p + "mask_token", (1, D), "zero", 0),
          (p + "patch_embed.proj.weight", (D, 3, PATCH, PATCH), "w", 3 * PATCH * PATCH),
          (p + "patch_embed.proj.bias", (D,), "b", 0)]
    for i in range(cfg["depth"]):
        b = f"{p}blocks.{i}."
        s += [(b + "norm1.weight", (D,), "g", 0), (b + "norm1.bias", (D,), "b", 0),
              (b + "attn.qkv.weight", (3 * D, D), "w", D), (b + "attn.qkv.bias", (3 * D,), "b", 0),
              (b + "attn.proj.weight", (D, D), "w", D), (b + "attn.proj.bias", (D,), "b", 0),
              (b + "ls1.gamma", (D,), "ls", 0),
              (b + "norm2.weight", (D,), "g", 0), (b + "norm2.bias", (D,), "b", 0),
              (b + "mlp.fc1.weight", (4 * D, D), "w", D), (b + "mlp.fc1.bias", (4 * D,), "b", 0),
              (b + "mlp.fc2.weight", (D, 4 * D), "w", 4 * D), (b + "mlp.fc2.bias", (D,), "b", 0),
              (b + "ls2.gamma", (D,), "ls", 0)]
    s += [(p + "norm.weight", (D,), "g", 0), (p + "norm.bias", (D,), "b", 0)]
    h = "depth_head."
    for i in range(4):
        s += [(f"{h}projects.{i}.weight", (oc[i], D, 1, 1), "w", D),
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
        for u in (1, 2):
            for c in (1, 2):
                s += [(f"{rb}resConfUnit{u}.conv{c}.weight", (F, F, 3, 3), "w", 9 * F),
                      (f"{rb}resConfUnit{u}.conv{c}.bias", (F,), "b", 0)]
    H2 = cfg["head_hidden"]
    s += [(h + "scratch.output_conv1.weight", (F // 2, F, 3, 3), "w", 9 * F),
          (h + "scratch.output_conv1.bias", (F // 2,), "b", 0),
          (h + "scratch.output_conv2.0.weight", (H2, F // 2, 3, 3), "w", 9 * (F // 2)),
          (h + "scratch.output_conv2.0.bias", (H2,), "b", 0),
          (h + "scratch.output_conv2.2.weight", (1, H2, 1, 1), "w", H2),
          (h + "scratch.output_conv2.2.bias", (1,), "b", 0)]
    return s


def synthetic_state_dict(cfg: dict, seed: int = 1234) -> "OrderedDict[str, np.ndarray]":
    """Seeded, fan-in scaled upstream-keyed state dict (float32 numpy)."""
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


def state_dict_digest(sd: Dict[str, np.ndarray]) -> str:
    """sha256 over keys + raw float32 bytes, in key order."""
    h = hashlib.sha256()
    for k in sorted(sd):
        a = np.ascontiguousarray(np.asarray(sd[k], dtype=np.float32))
        h.update(k.encode())
        h.update(str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


IMAGENET_MEAN = np.array([0.485, 0.456, 0.406], np.float64)
IMAGENET_STD = np.array([0.229, 0.224, 0.225], np.float64)


def synthetic_images_u8(batch: int, h: int = 518, w: int = 518, first_seed: int = 0) -> np.ndarray:
    """The same pixels as synthetic_images() before normalisation: uint8 NHWC
    [batch, h, w, 3] (the "image_u8" binding of a uint8_nhwc engine)."""
    out = np.empty((batch, h, w, 3), np.uint8)
    for i in range(batch):
        rng = np.random.Generator(np.random.PCG64(first_seed + i))
        out[i] = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
    return out


def synthetic_images(batch: int, h: int = 518, w: int = 518, first_seed: int = 0) -> np.ndarray:
    """The benchmark input domain: u ~ U{0..255} per pixel (PCG64 seed i for
    image i), then (u/255 - mean)/std in float64 -> float32 NCHW.  This is the
    tensor `core/preprocess.py` hands the engine (`models/depth_anything_v2/
    spec.json` input.normalize), minus the cv2 resize of a real photo."""
    out = np.empty((batch, 3, h, w), np.float32)
    for i in range(batch):
        rng = np.random.Generator(np.random.PCG64(first_seed + i))
        u = rng.integers(0, 256, size=(h, w, 3), dtype=np.uint8)
        x = (u.astype(np.float64) / 255.0 - IMAGENET_MEAN) / IMAGENET_STD
        out[i] = x.transpose(2, 0, 1).astype(np.float32)
    return out

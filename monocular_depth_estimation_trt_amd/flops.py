"""Algorithmic work of the DA-V2 forward, per layer (2 FLOP per MAC).

Counts the REFERENCE graph (upstream DepthAnythingV2 / the TensorRT engine
of SURVEY.md 2.3), not what the HIP schedule happens to execute: e.g. the
fusion out_conv is counted at the post-resize resolution even though the
engine runs it before the resize (4x fewer MACs, exact by linearity).  These
are the numbers roofline fractions are quoted against (ViT-S
115.27 GFLOP/img, ViT-L 1304.22 GFLOP/img at 518^2).

Layer names match the engine's profiler names (csrc/engine.hip Runner).
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict


def layer_flops(cfg: dict, img_h: int = 518, img_w: int = 518, batch: int = 1) -> "OrderedDict[str, float]":
    P = cfg["patch"]
    ph, pw = img_h // P, img_w // P
    npch = ph * pw
    T = npch + 1
    D, F = cfg["embed_dim"], cfg["features"]
    oc = cfg["out_channels"]
    M4 = cfg["mlp_hidden"]
    h4, w4 = (ph + 1) // 2, (pw + 1) // 2
    s = [(4 * ph) * (4 * pw), (2 * ph) * (2 * pw), npch, h4 * w4]
    o: "OrderedDict[str, float]" = OrderedDict()
    o["patch_embed"] = 2.0 * npch * D * 3 * P * P
    for i in range(cfg["depth"]):
        o[f"block{i}.qkv"] = 2.0 * T * 3 * D * D
        o[f"block{i}.attn"] = 4.0 * T * T * D
        o[f"block{i}.proj"] = 2.0 * T * D * D
        o[f"block{i}.fc1"] = 2.0 * T * M4 * D
        o[f"block{i}.fc2"] = 2.0 * T * D * M4
    for i in range(4):
        o[f"reassemble{i}.project"] = 2.0 * npch * D * oc[i]
    o["reassemble0.convT4"] = 2.0 * npch * oc[0] * oc[0] * 16
    o["reassemble1.convT2"] = 2.0 * npch * oc[1] * oc[1] * 4
    o["reassemble3.conv_s2"] = 2.0 * s[3] * oc[3] * oc[3] * 9
    for i in range(4):
        o[f"layer{i + 1}_rn"] = 2.0 * s[i] * F * oc[i] * 9
    # refinenet r works at scale index r-1; out_conv after the resize
    scale = {4: 3, 3: 2, 2: 1, 1: 0}
    target = {4: s[2], 3: s[1], 2: s[0], 1: 4 * s[0]}
    for r in (4, 3, 2, 1):
        px = s[scale[r]]
        units = (2,) if r == 4 else (1, 2)
        for u in units:
            o[f"rf{r}.rcu{u}.c1"] = 2.0 * px * F * F * 9
            o[f"rf{r}.rcu{u}.c2"] = 2.0 * px * F * F * 9
        o[f"rf{r}.out"] = 2.0 * target[r] * F * F
    H1 = (8 * ph) * (8 * pw)
    o["head.output_conv1"] = 2.0 * H1 * (F // 2) * F * 9
    o["head.output_conv2"] = 2.0 * img_h * img_w * (cfg["head_hidden"] * (F // 2) * 9 + cfg["head_hidden"])
    if batch != 1:
        for k in o:
            o[k] *= batch
    return o


def total_flops(cfg: dict, img_h: int = 518, img_w: int = 518, batch: int = 1) -> float:
    return float(sum(layer_flops(cfg, img_h, img_w, batch).values()))


def layer_class(name: str) -> str:
    """'block7.fc1' -> 'fc1'; 'rf3.rcu1.c2' -> 'rcu.conv'; others unchanged."""
    if name.startswith("block"):
        return name.split(".", 1)[1]
    if name.startswith("rf") and ".rcu" in name:
        return "rcu.conv"
    if name.startswith("rf") and name.endswith(".out"):
        return "fusion.out_conv"
    if name.startswith("rf") and name.endswith(".resize"):
        return "fusion.resize"
    if name.startswith("tap"):
        return "tap.norm"
    if name.startswith("layer") and name.endswith("_rn"):
        return "layer_rn"
    if name.startswith("reassemble") and name.endswith(".project"):
        return "reassemble.project"
    return name


def class_flops(cfg: dict, img_h: int = 518, img_w: int = 518, batch: int = 1) -> Dict[str, float]:
    out: Dict[str, float] = {}
    for k, v in layer_flops(cfg, img_h, img_w, batch).items():
        c = layer_class(k)
        out[c] = out.get(c, 0.0) + v
    return out

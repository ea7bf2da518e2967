"""Algorithmic work of the Depth Pro forward, per layer (2 FLOP per MAC).

Counts the REFERENCE graph (upstream apple/ml-depth-pro as restated by
HF:models/depth_pro/modeling_depth_pro.py), not what the HIP schedule
executes: each fusion layer's deconv(2,2) + 1x1 projection is counted as the
two layers it is in the reference even though the engine runs them as one
folded ConvT (half the MACs), and the FOV neck Linear is counted on all 577
tokens (cls included) as the reference applies it.

Layer names match the engine's profiler names (csrc/depth_pro.hip Runner).
"""

from __future__ import annotations

from collections import OrderedDict
from typing import Dict


def layer_flops(cfg: dict, batch: int = 1) -> "OrderedDict[str, float]":
    D, F, P = cfg["embed_dim"], cfg["fusion"], cfg["patch"]
    G = cfg["vit_size"] // P
    GG, T = G * G, G * G + 1
    M4 = cfg["mlp_hidden"]
    sd0, sd1, sd2 = cfg["scaled_dims"]
    id0, id1 = cfg["inter_dims"]
    S = cfg["img"]
    o: "OrderedDict[str, float]" = OrderedDict()
    encs = [("pe.", 35), ("ie.", 1)] + ([("fe.", 1)] if cfg["use_fov"] else [])
    for pfx, nseq in encs:
        o[pfx + "patch_embed"] = 2.0 * nseq * GG * D * 3 * P * P
        for i in range(cfg["depth"]):
            o[f"{pfx}block{i}.qkv"] = 2.0 * nseq * T * 3 * D * D
            o[f"{pfx}block{i}.attn"] = 4.0 * nseq * T * T * D
            o[f"{pfx}block{i}.proj"] = 2.0 * nseq * T * D * D
            o[f"{pfx}block{i}.fc1"] = 2.0 * nseq * T * M4 * D
            o[f"{pfx}block{i}.fc2"] = 2.0 * nseq * T * D * M4
    px = lambda k: float(k * k * GG)  # noqa: E731  pixels of a (k G)^2 map
    o["neck.image_block"] = 2.0 * px(1) * D * sd0 * 4
    o["neck.scaled0.proj"] = 2.0 * px(1) * D * sd0
    o["neck.scaled0.up"] = 2.0 * px(1) * sd0 * sd0 * 4
    o["neck.fuse_image_with_low_res"] = 2.0 * px(2) * 2 * sd0 * sd0
    o["neck.scaled1.proj"] = 2.0 * px(2) * D * sd1
    o["neck.scaled1.up"] = 2.0 * px(2) * sd1 * sd1 * 4
    o["neck.scaled2.proj"] = 2.0 * px(4) * D * sd2
    o["neck.scaled2.up"] = 2.0 * px(4) * sd2 * sd2 * 4
    o["neck.inter0.proj"] = 2.0 * px(4) * D * F
    o["neck.inter0.up0"] = 2.0 * px(4) * F * id0 * 4
    o["neck.inter0.up1"] = 2.0 * px(8) * id0 * id0 * 4
    o["neck.inter1.proj"] = 2.0 * px(4) * D * id1
    o["neck.inter1.up0"] = 2.0 * px(4) * id1 * id1 * 4
    o["neck.inter1.up1"] = 2.0 * px(8) * id1 * id1 * 4
    o["neck.inter1.up2"] = 2.0 * px(16) * id1 * id1 * 4
    for i, (k, cin) in enumerate(((2, sd0), (4, sd1), (8, sd2), (16, id0), (32, id1))):
        if i == 4 and cin == F:
            continue
        o[f"neck.projection{i}"] = 2.0 * px(k) * cin * F * 9
    for l in range(5):
        k = 2 << l
        for u in ((2,) if l == 0 else (1, 2)):
            for c in (1, 2):
                o[f"fs{l}.rcu{u}.c{c}"] = 2.0 * px(k) * F * F * 9
        if l < 4:
            o[f"fs{l}.up"] = 2.0 * px(k) * F * F * 4 + 2.0 * px(2 * k) * F * F   # deconv + projection
        else:
            o[f"fs{l}.out"] = 2.0 * px(k) * F * F
    o["head.conv1"] = 2.0 * px(32) * F * (F // 2) * 9
    o["head.deconv"] = 2.0 * px(32) * (F // 2) * (F // 2) * 4
    o["head.conv2_conv3"] = 2.0 * S * S * (cfg["head_hidden"] * (F // 2) * 9 + cfg["head_hidden"])
    if cfg["use_fov"]:
        o["fov.neck"] = 2.0 * T * D * (F // 2)
        o["fov.conv"] = 2.0 * GG * F * (F // 2) * 9
        o["fov.head0"] = 2.0 * (GG // 4) * (F // 2) * (F // 4) * 9
        o["fov.head1"] = 2.0 * (GG // 16) * (F // 4) * (F // 8) * 9
        o["fov.final"] = 2.0 * (GG // 16) * (F // 8)
    if batch != 1:
        for key in o:
            o[key] *= batch
    return o


def total_flops(cfg: dict, batch: int = 1) -> float:
    return float(sum(layer_flops(cfg, batch).values()))


def layer_class(name: str) -> str:
    """'pe.block7.fc1' -> 'pe.fc1'; 'fs3.rcu1.c2' -> 'fusion.rcu.conv'; 'neck.scaled1.up' -> 'neck.convT'."""
    parts = name.split(".")
    if len(parts) == 3 and parts[1].startswith("block"):
        return f"{parts[0]}.{parts[2]}"
    if name.startswith("fs") and ".rcu" in name:
        return "fusion.rcu.conv"
    if name.startswith("fs"):
        return "fusion.up" if name.endswith(".up") else "fusion.out"
    if name.startswith("neck.projection"):
        return "neck.projection"
    if name.startswith("neck.") and (name.endswith(".up") or ".up" in name[-4:] or name == "neck.image_block"):
        return "neck.convT"
    if name.startswith("neck.") and name.endswith(".proj"):
        return "neck.proj1x1"
    if name.endswith("merge") or ".merge" in name:
        return "merge"
    return name


def class_flops(cfg: dict, batch: int = 1) -> Dict[str, float]:
    out: Dict[str, float] = {}
    for k, v in layer_flops(cfg, batch).items():
        c = layer_class(k)
        out[c] = out.get(c, 0.0) + v
    return out

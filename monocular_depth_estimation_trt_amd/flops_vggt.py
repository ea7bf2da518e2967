"""Algorithmic work of the VGGT depth path, per layer (2 FLOP per MAC).

Counts the REFERENCE graph (`VGGTDepthOnlyWrapper`, models/vggt/onnx_export.py:
38-52: aggregator + depth head), not what the HIP schedule executes: the
fusion out_conv is counted after the resize although the engine runs it
before (exact by linearity), output_conv2's 1x1 is counted with both of its
output channels although the engine computes only the depth channel, and the
UV embedding convolution the packer folds into a table is not counted at all
(it is input-independent).  Global attention is counted over the whole
S * T sequence of each batch item.

Layer names match the engine's profiler names (csrc/vggt.hip Runner).
"""

from __future__ import annotations

import re
from collections import OrderedDict
from typing import Dict

NPRE = 5   # camera + 4 register tokens (aggregator); cls + 4 registers (DINOv2)


def layer_flops(cfg: dict, batch: int = 1, frames: int = 1) -> "OrderedDict[str, float]":
    P, Sz = cfg["patch"], cfg["img"]
    g = Sz // P
    npch = g * g
    T = npch + NPRE
    n = batch * frames                      # frames in the batch
    D, F = cfg["embed_dim"], cfg["features"]
    C2 = 2 * D
    oc = cfg["out_channels"]
    M4 = cfg["mlp_hidden"]
    h4 = (g + 1) // 2
    s = [(4 * g) ** 2, (2 * g) ** 2, npch, h4 * h4]
    o: "OrderedDict[str, float]" = OrderedDict()
    o["patch_embed"] = 2.0 * n * npch * D * 3 * P * P

    def block(pfx: str, seqs: int, L: int):
        o[pfx + ".qkv"] = 2.0 * seqs * L * 3 * D * D
        o[pfx + ".attn"] = 4.0 * seqs * L * L * D
        o[pfx + ".proj"] = 2.0 * seqs * L * D * D
        o[pfx + ".fc1"] = 2.0 * seqs * L * M4 * D
        o[pfx + ".fc2"] = 2.0 * seqs * L * D * M4

    for i in range(cfg["depth"]):
        block(f"db{i}", n, T)
    for i in range(cfg["aa_depth"]):
        block(f"fb{i}", n, T)
        block(f"gb{i}", batch, frames * T)
    for k in range(4):
        o[f"reassemble{k}.project"] = 2.0 * n * npch * C2 * oc[k]
    o["reassemble0.convT4"] = 2.0 * n * npch * oc[0] * oc[0] * 16
    o["reassemble1.convT2"] = 2.0 * n * npch * oc[1] * oc[1] * 4
    o["reassemble3.conv_s2"] = 2.0 * n * s[3] * oc[3] * oc[3] * 9
    for i in range(4):
        o[f"layer{i + 1}_rn"] = 2.0 * n * s[i] * F * oc[i] * 9
    scale = {4: 3, 3: 2, 2: 1, 1: 0}
    target = {4: s[2], 3: s[1], 2: s[0], 1: 4 * s[0]}
    for r in (4, 3, 2, 1):
        px = s[scale[r]]
        for u in ((2,) if r == 4 else (1, 2)):
            o[f"rf{r}.rcu{u}.c1"] = 2.0 * n * px * F * F * 9
            o[f"rf{r}.rcu{u}.c2"] = 2.0 * n * px * F * F * 9
        o[f"rf{r}.out"] = 2.0 * n * target[r] * F * F
    o["head.output_conv1"] = 2.0 * n * (8 * g) ** 2 * (F // 2) * F * 9
    o["head.output_conv2"] = 2.0 * n * Sz * Sz * (cfg["head_hidden"] * (F // 2) * 9 + cfg["head_hidden"] * 2)
    return o


def total_flops(cfg: dict, batch: int = 1, frames: int = 1) -> float:
    return float(sum(layer_flops(cfg, batch, frames).values()))


_BLK = re.compile(r"^(db|fb|gb)\d+\.(.+)$")


def layer_class(name: str) -> str:
    """'gb7.attn' -> 'gb.attn'; 'rf3.rcu1.c2' -> 'rcu.conv'; others as flops.layer_class."""
    m = _BLK.match(name)
    if m:
        return f"{m.group(1)}.{m.group(2)}"
    from .flops import layer_class as dav2_class
    return dav2_class(name)


def class_flops(cfg: dict, batch: int = 1, frames: int = 1) -> Dict[str, float]:
    out: Dict[str, float] = {}
    for k, v in layer_flops(cfg, batch, frames).items():
        c = layer_class(k)
        out[c] = out.get(c, 0.0) + v
    return out

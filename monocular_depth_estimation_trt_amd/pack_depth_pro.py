"""AOT weight packer for Depth Pro: HF-keyed state dict -> packed engine.

Replaces the reference's `models/depth_pro/onnx_export.py:13-60` (ONNX
opset 20, dynamo export of apple/ml-depth-pro at its fixed 1536x1536 input)
and the TensorRT build of `core/common.py:get_engine` for this model.  Same
container as pack.py (csrc/pack_format.h) with `family = 1`; the layouts:

* three DINOv2 encoders under "pe." (patch), "ie." (image), "fe." (fov):
  patch-embed [D][3*16*16], fused qkv rows [q; k; v] (HF splits them),
  pos table without the cls row + cls folded with pos[0];
* 1x1 convs / Linear -> f16 [Npad][Kpad]; 3x3 convs -> [Cout][ky][kx][Cin];
  ConvTranspose(2, 2) -> [(dy*2+dx)*Cout+co][Cin] (GEMM + pixel-shuffle);
* every fusion layer's deconv(2,2) and the 1x1 projection after it are
  folded into ONE ConvTranspose weight (W'[ci][co] = sum_c Wp[co][c] Wt[ci][c],
  bias = the projection's): both are linear per output pixel, and the fold
  removes a full 1x1 pass at 4x the resolution (96^2 .. 768^2 x 256);
* the FOV head's last valid 6x6 conv -> fp32 [ky][kx][c] for a dot product.

Key names: transformers' DepthProForDepthEstimation (the `apple/DepthPro-hf`
checkpoint layout, weights_depth_pro.py).
"""

from __future__ import annotations

import struct
from collections import OrderedDict
from typing import Dict

import numpy as np

from . import pack as PK
from . import weights_depth_pro as WD

FAMILY_DEPTH_PRO = 1


def _vit(o, sd, src: str, dst: str, cfg: dict):
    D, P = cfg["embed_dim"], cfg["patch"]
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1)  # noqa: E731
    e = src + "embeddings."
    o[dst + "patch.w"] = PK._pad2(sd[e + "patch_embeddings.projection.weight"].reshape(D, 3 * P * P))
    o[dst + "patch.b"] = f32(sd[e + "patch_embeddings.projection.bias"])
    pos = sd[e + "position_embeddings"]
    o[dst + "pos.patch"] = np.ascontiguousarray(pos[0, 1:], dtype=np.float32)
    o[dst + "pos.cls"] = f32(sd[e + "cls_token"].reshape(-1) + pos[0, 0])
    for i in range(cfg["depth"]):
        b = f"{src}encoder.layer.{i}."
        a = b + "attention.attention."
        q = f"{dst}b{i}."
        o[q + "ln1.g"] = f32(sd[b + "norm1.weight"])
        o[q + "ln1.b"] = f32(sd[b + "norm1.bias"])
        o[q + "qkv.w"] = PK._pad2(np.concatenate([sd[a + n + ".weight"] for n in ("query", "key", "value")], 0))
        o[q + "qkv.b"] = f32(np.concatenate([sd[a + n + ".bias"] for n in ("query", "key", "value")], 0))
        o[q + "proj.w"] = PK._pad2(sd[b + "attention.output.dense.weight"])
        o[q + "proj.b"] = f32(sd[b + "attention.output.dense.bias"])
        o[q + "ls1"] = f32(sd[b + "layer_scale1.lambda1"])
        o[q + "ln2.g"] = f32(sd[b + "norm2.weight"])
        o[q + "ln2.b"] = f32(sd[b + "norm2.bias"])
        o[q + "fc1.w"] = PK._pad2(sd[b + "mlp.fc1.weight"])
        o[q + "fc1.b"] = f32(sd[b + "mlp.fc1.bias"])
        o[q + "fc2.w"] = PK._pad2(sd[b + "mlp.fc2.weight"])
        o[q + "fc2.b"] = f32(sd[b + "mlp.fc2.bias"])
        o[q + "ls2"] = f32(sd[b + "layer_scale2.lambda1"])
    o[dst + "norm.g"] = f32(sd[src + "layernorm.weight"])
    o[dst + "norm.b"] = f32(sd[src + "layernorm.bias"])


def _1x1(w: np.ndarray) -> np.ndarray:
    return PK._pad2(w.reshape(w.shape[0], -1))


def fold_deconv_projection(wt: np.ndarray, wp: np.ndarray) -> np.ndarray:
    """ConvT weight [Cin][C][2][2] followed by a 1x1 conv [Co][C][1][1] ->
    one ConvT weight [Cin][Co][2][2] (fp64 accumulation)."""
    return np.einsum("oc,icyx->ioyx", wp.reshape(wp.shape[0], -1).astype(np.float64),
                     wt.astype(np.float64)).astype(np.float32)


def packed_tensors(sd: Dict[str, np.ndarray], cfg: dict) -> "OrderedDict[str, np.ndarray]":
    sd = PK.normalize_keys(sd)
    missing = [k for k in WD.expected_keys(cfg) if k not in sd and not k.endswith("mask_token")]
    if missing:
        raise KeyError(f"Depth Pro state dict lacks {len(missing)} keys, e.g. {missing[:4]}")
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1)  # noqa: E731
    o: "OrderedDict[str, np.ndarray]" = OrderedDict()
    _vit(o, sd, "depth_pro.encoder.patch_encoder.model.", "pe.", cfg)
    _vit(o, sd, "depth_pro.encoder.image_encoder.model.", "ie.", cfg)
    if cfg["use_fov"]:
        _vit(o, sd, "fov_model.fov_encoder.model.", "fe.", cfg)
    u = "depth_pro.neck.feature_upsample."
    o["img.up.w"] = PK._convT(sd[u + "image_block.layers.0.weight"])
    o["img.up.b"] = f32(sd[u + "image_block.layers.0.bias"])
    for i in range(len(cfg["scaled_dims"])):
        o[f"s{i}.proj.w"] = _1x1(sd[f"{u}scaled_images.{i}.layers.0.weight"])
        o[f"s{i}.up.w"] = PK._convT(sd[f"{u}scaled_images.{i}.layers.1.weight"])
    for i in range(len(cfg["inter_dims"])):
        o[f"h{i}.proj.w"] = _1x1(sd[f"{u}intermediate.{i}.layers.0.weight"])
        for j in range(2 + i):
            o[f"h{i}.up{j}.w"] = PK._convT(sd[f"{u}intermediate.{i}.layers.{j + 1}.weight"])
    n = "depth_pro.neck."
    o["fuse.w"] = _1x1(sd[n + "fuse_image_with_low_res.weight"])
    o["fuse.b"] = f32(sd[n + "fuse_image_with_low_res.bias"])
    for i in range(5):
        k = f"{n}feature_projection.projections.{i}.weight"
        if k in sd:
            o[f"prj{i}.w"] = PK._conv3(sd[k])
    nl = len(cfg["hooks"]) + len(cfg["ratios"])
    for i in range(nl):
        src = f"fusion_stage.intermediate.{i}." if i < nl - 1 else "fusion_stage.final."
        dst = f"fs{i}."
        for ru in (1, 2):
            if i == 0 and ru == 1:
                continue  # the first fusion layer never sees a residual input
            for c in (1, 2):
                o[f"{dst}rcu{ru}.c{c}.w"] = PK._conv3(sd[f"{src}residual_layer{ru}.convolution{c}.weight"])
                o[f"{dst}rcu{ru}.c{c}.b"] = f32(sd[f"{src}residual_layer{ru}.convolution{c}.bias"])
        if i < nl - 1:
            o[dst + "up.w"] = PK._convT(fold_deconv_projection(sd[src + "deconv.weight"], sd[src + "projection.weight"]))
            o[dst + "up.b"] = f32(sd[src + "projection.bias"])
        else:
            o[dst + "out.w"] = _1x1(sd[src + "projection.weight"])
            o[dst + "out.b"] = f32(sd[src + "projection.bias"])
    o["head.c1.w"] = PK._conv3(sd["head.layers.0.weight"])
    o["head.c1.b"] = f32(sd["head.layers.0.bias"])
    o["head.up.w"] = PK._convT(sd["head.layers.1.weight"])
    o["head.up.b"] = f32(sd["head.layers.1.bias"])
    o["head.c2.w"] = PK._conv3(sd["head.layers.2.weight"])
    o["head.c2.b"] = f32(sd["head.layers.2.bias"])
    o["head.c3.w"] = f32(sd["head.layers.4.weight"])
    o["head.c3.b"] = f32(sd["head.layers.4.bias"])
    if cfg["use_fov"]:
        fv = "fov_model."
        o["fov.neck.w"] = PK._pad2(sd[fv + "fov_encoder.neck.weight"])
        o["fov.neck.b"] = f32(sd[fv + "fov_encoder.neck.bias"])
        o["fov.conv.w"] = PK._conv3(sd[fv + "conv.weight"])
        o["fov.conv.b"] = f32(sd[fv + "conv.bias"])
        for i in range(cfg["fov_layers"]):
            o[f"fov.h{i}.w"] = PK._conv3(sd[f"{fv}head.layers.{2 * i}.weight"])
            o[f"fov.h{i}.b"] = f32(sd[f"{fv}head.layers.{2 * i}.bias"])
        L = 2 * cfg["fov_layers"]
        o["fov.final.w"] = f32(sd[f"{fv}head.layers.{L}.weight"][0].transpose(1, 2, 0))  # [c][k][k] -> [k][k][c]
        o["fov.final.b"] = f32(sd[f"{fv}head.layers.{L}.bias"])
    return o


def config_bytes(cfg: dict) -> bytes:
    """PackConfig (csrc/pack_format.h) with family = 1 and the Depth Pro geometry."""
    S = cfg["img"]
    b = struct.pack("<8i4i4i2i2f16s", cfg["embed_dim"], cfg["depth"], cfg["num_heads"], cfg["mlp_hidden"],
                    cfg["patch"], S, S, cfg["fusion"], 0, 0, 0, 0, 0, 0, 0, 0, cfg["head_hidden"], 0, 0.0,
                    float(cfg["ln_eps"]), cfg["encoder"].encode()[:15])
    b += struct.pack("<if3f3f", 0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    assert len(b) == 128, len(b)
    hooks, idims, sdims = cfg["hooks"], cfg["inter_dims"], cfg["scaled_dims"]
    if len(hooks) != 2 or len(idims) != 2 or len(sdims) != 3 or list(cfg["ratios"]) != [0.25, 0.5, 1.0] \
            or list(cfg["overlaps"]) != [0.0, 0.5, 0.25]:
        raise ValueError("the packed engine supports the upstream Depth Pro pyramid / hook layout only")
    b += struct.pack("<6i2i2i3i", FAMILY_DEPTH_PRO, cfg["vit_size"], cfg["merge_pad"], 1 if cfg["use_fov"] else 0,
                     cfg["fov_layers"], WD.fov_final_kernel(cfg), *hooks, *idims, *sdims)
    assert len(b) == 180, len(b)
    return b + b"\0" * 76


def pack_bytes(sd: Dict[str, np.ndarray], cfg: dict) -> bytes:
    return PK.container(packed_tensors(sd, cfg), config_bytes(cfg))


def synthetic_blob(preset: str = "dinov2l16_384", use_fov: bool = True, seed: int = 4321):
    cfg = WD.depth_pro_config(preset, use_fov=use_fov)
    return pack_bytes(WD.synthetic_state_dict(cfg, seed), cfg), cfg

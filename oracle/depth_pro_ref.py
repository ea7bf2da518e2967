"""ORACLE -- test infrastructure only.  CPU fp32 restatement of the Depth Pro
forward pass (three DINOv2-L/16 encoders at 384^2, the multi-resolution
patch pyramid, the upsampling neck, the deconv fusion stage, the depth head
and the FOV head).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker / the reported CPU baseline.  The
product path (`monocular_depth_estimation_trt_amd`) never calls it.

What it restates.  The reference runs Depth Pro as a TensorRT engine built
from an ONNX export of apple/ml-depth-pro (`models/depth_pro/onnx_export.py:
13-60`, outputs "canonical_inverse_depth" and "fov_deg"), driven by
`models/depth_pro/onnx2trt.py:42-125`.  The upstream repository is not
vendored (cloned at run time, no pin: `models/depth_pro/README.md` setup), so
the arithmetic follows the in-container transformers port line by line
(`HF:` = transformers 5.15.0 models/depth_pro/modeling_depth_pro.py):

* pyramid: bilinear(align_corners=False) x0.25 / x0.5 / x1     -- HF:238-262
* split into 384^2 patches, stride 384*(1-overlap), unfold order -- HF:74-88, 264-272
* DINOv2 encoder (patch 16, cls, pos, pre-LN blocks, LayerScale,
  final LayerNorm; hooks = raw block outputs)                   -- HF:274-333 + models/dinov2
* reconstruct: drop cls, 24x24 grid, merge with `merge_pad / ratio`
  rows/cols trimmed on interior edges, bilinear to the base size -- HF:91-217
* neck: per-scale 1x1 proj + ConvT(2,2) stacks, image ConvT,
  cat + 1x1 fuse, 3x3 projections (no bias)                      -- HF:441-600
* fusion stage: pre-act residual units, deconv(2,2) + 1x1 projection,
  final layer without deconv                                     -- HF:699-832
* head: conv3 -> ConvT(2,2) -> conv3 -> ReLU -> conv1 -> ReLU    -- HF:951-992
* FOV: encoder + Linear neck, conv3 s2 + ReLU on the global features, add,
  2 x (conv3 s2 + ReLU), final valid conv -> degrees            -- HF:835-948

Parity: pinned against `DepthProForDepthEstimation` built from a local config
by `tests/golden/make_golden_depth_pro.py` (fixtures under tests/golden/).
The reference publishes no vectors for this path, so that HF
cross-check is the pin.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["forward", "to_torch", "dinov2", "pyramid_patches", "merge", "patch_grid"]


def to_torch(sd: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)).float() for k, v in sd.items()}


def patch_grid(img: int, vit: int, ratio: float, overlap: float) -> Tuple[int, int, int]:
    """(scaled size, patches per side, stride) of one pyramid level."""
    s = int(img * ratio)
    if s == vit:
        return s, 1, vit
    stride = int(vit * (1 - overlap))
    n = (s - vit) // stride + 1
    return s, n, stride


def pyramid_patches(x: torch.Tensor, cfg: dict) -> Tuple[torch.Tensor, List[int]]:
    """The patch encoder's input: [sum_l n_l^2 * B, 3, vit, vit], high-res
    level first, patch-major / batch-minor (F.unfold order), and the per-level
    patch counts low-res first."""
    vit = cfg["vit_size"]
    levels = []
    for r, ov in zip(cfg["ratios"], cfg["overlaps"]):
        xs = x if r == 1 else F.interpolate(x, scale_factor=r, mode="bilinear", align_corners=False)
        s, n, stride = patch_grid(x.shape[-1], vit, r, ov)
        if n == 1 and s == vit:
            levels.append(xs)
            continue
        B, C = xs.shape[:2]
        p = F.unfold(xs, kernel_size=(vit, vit), stride=(stride, stride))       # [B, C*vit*vit, L]
        levels.append(p.permute(2, 0, 1).reshape(-1, C, vit, vit))
    counts = [len(t) for t in levels]
    return torch.cat(levels[::-1], 0), counts


def dinov2(w: Dict[str, torch.Tensor], pfx: str, cfg: dict, x: torch.Tensor,
           hooks=()) -> Tuple[torch.Tensor, Dict[int, torch.Tensor]]:
    """DINOv2 encoder (HF naming).  Returns (final-LayerNorm tokens
    [N, 1+G*G, D], {hook: raw block output})."""
    D, nh, P = cfg["embed_dim"], cfg["num_heads"], cfg["patch"]
    dh = D // nh
    eps = cfg["ln_eps"]
    e = pfx + "embeddings."
    N = x.shape[0]
    t = F.conv2d(x, w[e + "patch_embeddings.projection.weight"], w[e + "patch_embeddings.projection.bias"], stride=P)
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat([w[e + "cls_token"].expand(N, -1, -1), t], 1) + w[e + "position_embeddings"]
    T = t.shape[1]
    raw = {}
    for i in range(cfg["depth"]):
        b = f"{pfx}encoder.layer.{i}."
        a = f"{b}attention.attention."
        h = F.layer_norm(t, (D,), w[b + "norm1.weight"], w[b + "norm1.bias"], eps)
        q = F.linear(h, w[a + "query.weight"], w[a + "query.bias"]).reshape(N, T, nh, dh).transpose(1, 2)
        k = F.linear(h, w[a + "key.weight"], w[a + "key.bias"]).reshape(N, T, nh, dh).transpose(1, 2)
        v = F.linear(h, w[a + "value.weight"], w[a + "value.bias"]).reshape(N, T, nh, dh).transpose(1, 2)
        att = ((q @ k.transpose(-2, -1)) * (dh ** -0.5)).softmax(-1)
        o = (att @ v).transpose(1, 2).reshape(N, T, D)
        o = F.linear(o, w[b + "attention.output.dense.weight"], w[b + "attention.output.dense.bias"])
        t = t + w[b + "layer_scale1.lambda1"] * o
        h = F.layer_norm(t, (D,), w[b + "norm2.weight"], w[b + "norm2.bias"], eps)
        h = F.linear(F.gelu(F.linear(h, w[b + "mlp.fc1.weight"], w[b + "mlp.fc1.bias"])),
                     w[b + "mlp.fc2.weight"], w[b + "mlp.fc2.bias"])
        t = t + w[b + "layer_scale2.lambda1"] * h
        if i in hooks:
            raw[i] = t
    return F.layer_norm(t, (D,), w[pfx + "layernorm.weight"], w[pfx + "layernorm.bias"], eps), raw


def _grid(tokens: torch.Tensor) -> torch.Tensor:
    """drop cls, [N, T, C] -> [N, C, G, G]"""
    N, T, C = tokens.shape
    G = int(math.isqrt(T - 1))
    return tokens[:, -G * G:].reshape(N, G, G, C).permute(0, 3, 1, 2)


def merge(maps: torch.Tensor, B: int, pad: int) -> torch.Tensor:
    """Patch maps [n*n*B, C, G, G] (patch-major) -> [B, C, n*G - 2(n-1)pad, ...]:
    interior edges lose `pad` rows/cols (HF merge_patches)."""
    n2 = maps.shape[0] // B
    n = int(math.isqrt(n2))
    if n2 == 1:
        return maps
    G = maps.shape[-1]
    if n2 < 4:
        pad = 0
    pad = min(G // 4, pad)
    rows = []
    for r in range(n):
        cols = []
        for c in range(n):
            box = maps[B * (r * n + c):B * (r * n + c + 1)]
            t0 = pad if r else 0
            b0 = G - pad if r != n - 1 else G
            l0 = pad if c else 0
            r0 = G - pad if c != n - 1 else G
            cols.append(box[:, :, t0:b0, l0:r0])
        rows.append(torch.cat(cols, -1))
    return torch.cat(rows, -2)


def _reconstruct(tokens, B, pad, size):
    m = merge(_grid(tokens), B, pad)
    return F.interpolate(m, size=size, mode="bilinear", align_corners=False)


def _upsample_block(w, pfx, x, n_layers, proj=True, bias=False):
    j = 0
    if proj:
        x = F.conv2d(x, w[f"{pfx}layers.0.weight"])
        j = 1
    for i in range(n_layers):
        k = f"{pfx}layers.{j + i}."
        x = F.conv_transpose2d(x, w[k + "weight"], w.get(k + "bias") if bias else None, stride=2)
    return x


def _rcu(w, pfx, x):
    o = F.conv2d(F.relu(x), w[pfx + "convolution1.weight"], w[pfx + "convolution1.bias"], padding=1)
    o = F.conv2d(F.relu(o), w[pfx + "convolution2.weight"], w[pfx + "convolution2.bias"], padding=1)
    return o + x


def _fusion_layer(w, pfx, h, res=None, deconv=True):
    if res is not None:
        h = h + _rcu(w, pfx + "residual_layer1.", res)
    h = _rcu(w, pfx + "residual_layer2.", h)
    if deconv:
        h = F.conv_transpose2d(h, w[pfx + "deconv.weight"], None, stride=2)
    return F.conv2d(h, w[pfx + "projection.weight"], w[pfx + "projection.bias"])


@torch.no_grad()
def forward(w: Dict[str, torch.Tensor], cfg: dict, x, keep: Optional[dict] = None
            ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """DepthProForDepthEstimation.forward: x float32 NCHW [B,3,1536,1536]
    (normalised to [-1, 1]) -> (canonical inverse depth [B, 1536, 1536],
    fov degrees [B] or None)."""
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(x)
    x = x.float()
    B, _, H, W_ = x.shape
    vit, P = cfg["vit_size"], cfg["patch"]
    G = vit // P
    exp = int(math.log2(W_ / G))
    bh, bw = H // 2 ** exp, W_ // 2 ** exp
    # ---- encoders ----
    patches, counts = pyramid_patches(x, cfg)
    pe = "depth_pro.encoder.patch_encoder.model."
    last, raw = dinov2(w, pe, cfg, patches, hooks=cfg["hooks"])
    per_level = list(torch.split(last, counts[::-1]))[::-1]     # low-res first
    feats_scaled = []
    for i, (r, t) in enumerate(zip(cfg["ratios"], per_level)):
        pad = int(cfg["merge_pad"] * (1 / r))
        feats_scaled.append(_reconstruct(t, B, pad, (bh * 2 ** i, bw * 2 ** i)))
    nhi = counts[-1]
    feats_inter = []
    for hk in cfg["hooks"]:
        pad = int(cfg["merge_pad"] * (1 / cfg["ratios"][-1]))
        n = len(cfg["ratios"]) - 1
        feats_inter.append(_reconstruct(raw[hk][:nhi], B, pad, (bh * 2 ** n, bw * 2 ** n)))
    xi = F.interpolate(x, size=(vit, vit), mode="bilinear", align_corners=False)
    img_tok, _ = dinov2(w, "depth_pro.encoder.image_encoder.model.", cfg, xi)
    feat_img = _reconstruct(img_tok, B, 0, (bh, bw))
    # ---- neck ----
    u = "depth_pro.neck.feature_upsample."
    f0 = _upsample_block(w, u + "image_block.", feat_img, 1, proj=False, bias=True)
    fs = [_upsample_block(w, f"{u}scaled_images.{i}.", f, 1) for i, f in enumerate(feats_scaled)]
    fi = [_upsample_block(w, f"{u}intermediate.{i}.", f, 2 + i) for i, f in enumerate(feats_inter)]
    g = torch.cat([fs[0], f0], 1)
    g = F.conv2d(g, w["depth_pro.neck.fuse_image_with_low_res.weight"], w["depth_pro.neck.fuse_image_with_low_res.bias"])
    feats = [g, *fs[1:], *fi]
    proj = []
    for i, f in enumerate(feats):
        k = f"depth_pro.neck.feature_projection.projections.{i}.weight"
        proj.append(F.conv2d(f, w[k], padding=1) if k in w else f)
    # ---- fusion stage ----
    nl = len(proj)
    h = None
    for i in range(nl - 1):
        h = _fusion_layer(w, f"fusion_stage.intermediate.{i}.", proj[i] if h is None else h,
                          None if h is None else proj[i])
    h = _fusion_layer(w, "fusion_stage.final.", h, proj[-1], deconv=False)
    # ---- head ----
    o = F.conv2d(h, w["head.layers.0.weight"], w["head.layers.0.bias"], padding=1)
    o = F.conv_transpose2d(o, w["head.layers.1.weight"], w["head.layers.1.bias"], stride=2)
    o = F.relu(F.conv2d(o, w["head.layers.2.weight"], w["head.layers.2.bias"], padding=1))
    depth = F.relu(F.conv2d(o, w["head.layers.4.weight"], w["head.layers.4.bias"])).squeeze(1)
    if keep is not None:
        keep.update(proj=proj, fused=h, feats_scaled=feats_scaled, feats_inter=feats_inter, feat_img=feat_img)
    fov = None
    if cfg["use_fov"]:
        fv = "fov_model."
        ft, _ = dinov2(w, fv + "fov_encoder.model.", cfg, xi)
        ft = F.linear(ft, w[fv + "fov_encoder.neck.weight"], w[fv + "fov_encoder.neck.bias"])
        ff = _reconstruct(ft, B, 0, (bh, bw))
        gl = F.relu(F.conv2d(proj[0], w[fv + "conv.weight"], w[fv + "conv.bias"], stride=2, padding=1))
        z = F.interpolate(ff + gl, size=(G, G), mode="bilinear", align_corners=False)
        for i in range(cfg["fov_layers"]):
            k = f"{fv}head.layers.{2 * i}."
            z = F.relu(F.conv2d(z, w[k + "weight"], w[k + "bias"], stride=2, padding=1))
        k = f"{fv}head.layers.{2 * cfg['fov_layers']}."
        fov = F.conv2d(z, w[k + "weight"], w[k + "bias"]).flatten()
    return depth, fov

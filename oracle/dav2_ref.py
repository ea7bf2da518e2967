"""ORACLE -- test infrastructure only.  CPU fp32 restatement of the Depth
Anything V2 forward pass (DINOv2 ViT encoder + DPT head).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker / the reported CPU baseline.  The
product path (`monocular_depth_estimation_trt_amd`) never calls it.

What it restates.  The reference runs this graph inside TensorRT, compiled
from an ONNX export of the *upstream* PyTorch model
(`models/depth_anything_v2/onnx_export.py:19-66`, model built by
`models/depth_anything_v2/infer_metric.py:53-68`).  The upstream repository is
not vendored in the reference (cloned at run time, no version pin:
`models/depth_anything_v2/infer.py:13-15`), so the arithmetic below follows
its published structure, with the in-container HF port as the line-by-line
cross-check (`HF:` = transformers 5.15.0 under site-packages):

* patch embed Conv2d(3, D, 14, s14) -- HF:models/dinov2/modeling_dinov2.py:139-148
* cls concat + pos embed (+ upstream bicubic interpolation with the 0.1 offset
  when the grid differs from 37x37)   -- HF:.../modeling_dinov2.py:57-116
* 12/24 pre-LN blocks, LayerScale      -- HF:.../modeling_dinov2.py:342-381
* taps after blocks [2,5,8,11] / [4,11,17,23] with the final norm applied
  (get_intermediate_layers(norm=True)) -- HF:.../modeling_dinov2.py:598-608
* DPT reassemble / fusion / head       -- HF:models/depth_anything/
  modeling_depth_anything.py:31-306 (HF's fusion list is upstream's
  refinenet4..1 reversed)
* metric head: Sigmoid * max_depth (infer_metric.py:61-66); relative: ReLU.

Parity: pinned against `DepthAnythingForDepthEstimation` by
`tests/golden/make_golden.py` (fixtures under tests/golden/, checked by
tests/test_oracle_golden.py).  The reference itself publishes no vectors for
this path, so that HF cross-check is the pin.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["forward", "interpolate_pos_embed", "to_torch", "encoder_taps", "dpt_head",
           "bilinear_ac"]


def to_torch(sd: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)).float() for k, v in sd.items()}


def interpolate_pos_embed(pos_embed: torch.Tensor, ph: int, pw: int) -> torch.Tensor:
    """Upstream DINOv2 `interpolate_pos_encoding` (interpolate_offset=0.1,
    antialias False, bicubic).  pos_embed [1, 1+M*M, D] -> [1, 1+ph*pw, D]."""
    N = pos_embed.shape[1] - 1
    if N == ph * pw and ph == pw:
        return pos_embed
    M = int(math.sqrt(N))
    assert M * M == N
    D = pos_embed.shape[-1]
    cls = pos_embed[:, :1].float()
    patch = pos_embed[:, 1:].float().reshape(1, M, M, D).permute(0, 3, 1, 2)
    sx = float(ph + 0.1) / M
    sy = float(pw + 0.1) / M
    patch = F.interpolate(patch, scale_factor=(sx, sy), mode="bicubic", antialias=False)
    assert tuple(patch.shape[-2:]) == (ph, pw), patch.shape
    patch = patch.permute(0, 2, 3, 1).reshape(1, ph * pw, D)
    return torch.cat([cls, patch], dim=1)


def encoder_taps(w: Dict[str, torch.Tensor], cfg: dict, x: torch.Tensor) -> List[torch.Tensor]:
    """DINOv2 forward; returns the 4 normed tap token maps [B, 1+ph*pw, D]."""
    B, _, H, W = x.shape
    P = cfg["patch"]
    ph, pw = H // P, W // P
    D, nh = cfg["embed_dim"], cfg["num_heads"]
    dh = D // nh
    eps = cfg["ln_eps"]
    p = "pretrained."
    t = F.conv2d(x, w[p + "patch_embed.proj.weight"], w[p + "patch_embed.proj.bias"], stride=P)
    t = t.flatten(2).transpose(1, 2)                                     # [B, ph*pw, D]
    t = torch.cat([w[p + "cls_token"].expand(B, -1, -1), t], dim=1)
    t = t + interpolate_pos_embed(w[p + "pos_embed"], ph, pw)
    T = t.shape[1]
    taps = []
    for i in range(cfg["depth"]):
        b = f"{p}blocks.{i}."
        h = F.layer_norm(t, (D,), w[b + "norm1.weight"], w[b + "norm1.bias"], eps)
        qkv = F.linear(h, w[b + "attn.qkv.weight"], w[b + "attn.qkv.bias"])
        qkv = qkv.reshape(B, T, 3, nh, dh).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0] * (dh ** -0.5), qkv[1], qkv[2]
        a = (q @ k.transpose(-2, -1)).softmax(dim=-1)
        o = (a @ v).transpose(1, 2).reshape(B, T, D)
        o = F.linear(o, w[b + "attn.proj.weight"], w[b + "attn.proj.bias"])
        t = t + w[b + "ls1.gamma"] * o
        h = F.layer_norm(t, (D,), w[b + "norm2.weight"], w[b + "norm2.bias"], eps)
        h = F.linear(h, w[b + "mlp.fc1.weight"], w[b + "mlp.fc1.bias"])
        h = F.gelu(h)
        h = F.linear(h, w[b + "mlp.fc2.weight"], w[b + "mlp.fc2.bias"])
        t = t + w[b + "ls2.gamma"] * h
        if i in cfg["taps"]:
            taps.append(F.layer_norm(t, (D,), w[p + "norm.weight"], w[p + "norm.bias"], eps))
    return taps


def bilinear_ac(x: torch.Tensor, size) -> torch.Tensor:
    return F.interpolate(x, size=tuple(int(s) for s in size), mode="bilinear", align_corners=True)


def _rcu(w, pre, x):
    """ResidualConvUnit (pre-activation, bias, bn=False)."""
    o = F.relu(x)
    o = F.conv2d(o, w[pre + "conv1.weight"], w[pre + "conv1.bias"], padding=1)
    o = F.relu(o)
    o = F.conv2d(o, w[pre + "conv2.weight"], w[pre + "conv2.bias"], padding=1)
    return o + x


def _fusion(w, pre, x0, x1=None, size=None):
    """FeatureFusionBlock(deconv=False, expand=False, align_corners=True)."""
    out = x0
    if x1 is not None:
        out = out + _rcu(w, pre + "resConfUnit1.", x1)
    out = _rcu(w, pre + "resConfUnit2.", out)
    if size is None:
        size = (out.shape[2] * 2, out.shape[3] * 2)
    out = bilinear_ac(out, size)
    return F.conv2d(out, w[pre + "out_conv.weight"], w[pre + "out_conv.bias"])


def dpt_head(w: Dict[str, torch.Tensor], cfg: dict, taps: List[torch.Tensor], ph: int, pw: int,
             keep: Optional[dict] = None) -> torch.Tensor:
    """DPTHead.forward (use_clstoken=False) + the model's final activation.
    Returns depth [B, ph*14, pw*14]."""
    h = "depth_head."
    B = taps[0].shape[0]
    feats = []
    for i, t in enumerate(taps):
        t = t[:, 1:]                                                       # drop cls
        t = t.permute(0, 2, 1).reshape(B, t.shape[-1], ph, pw)
        t = F.conv2d(t, w[f"{h}projects.{i}.weight"], w[f"{h}projects.{i}.bias"])
        if i == 0:
            t = F.conv_transpose2d(t, w[h + "resize_layers.0.weight"], w[h + "resize_layers.0.bias"], stride=4)
        elif i == 1:
            t = F.conv_transpose2d(t, w[h + "resize_layers.1.weight"], w[h + "resize_layers.1.bias"], stride=2)
        elif i == 3:
            t = F.conv2d(t, w[h + "resize_layers.3.weight"], w[h + "resize_layers.3.bias"], stride=2, padding=1)
        feats.append(t)
    rn = [F.conv2d(f, w[f"{h}scratch.layer{i + 1}_rn.weight"], None, padding=1) for i, f in enumerate(feats)]
    s = h + "scratch."
    p4 = _fusion(w, s + "refinenet4.", rn[3], size=rn[2].shape[2:])
    p3 = _fusion(w, s + "refinenet3.", p4, rn[2], size=rn[1].shape[2:])
    p2 = _fusion(w, s + "refinenet2.", p3, rn[1], size=rn[0].shape[2:])
    p1 = _fusion(w, s + "refinenet1.", p2, rn[0])
    o = F.conv2d(p1, w[s + "output_conv1.weight"], w[s + "output_conv1.bias"], padding=1)
    o = bilinear_ac(o, (ph * cfg["patch"], pw * cfg["patch"]))
    o = F.conv2d(o, w[s + "output_conv2.0.weight"], w[s + "output_conv2.0.bias"], padding=1)
    o = F.relu(o)
    o = F.conv2d(o, w[s + "output_conv2.2.weight"], w[s + "output_conv2.2.bias"])
    if keep is not None:
        keep.update(feats=feats, rn=rn, paths=[p4, p3, p2, p1])
    if cfg["depth_type"] == "metric":
        o = torch.sigmoid(o) * cfg["max_depth"]
    else:
        o = F.relu(F.relu(o))
    return o.squeeze(1)


@torch.no_grad()
def forward(w: Dict[str, torch.Tensor], cfg: dict, x, keep: Optional[dict] = None) -> torch.Tensor:
    """DepthAnythingV2.forward: x float32 NCHW [B,3,H,W] (H, W multiples of 14)
    -> depth float32 [B, H, W]."""
    if isinstance(x, np.ndarray):
        x = torch.from_numpy(x)
    x = x.float()
    P = cfg["patch"]
    ph, pw = x.shape[-2] // P, x.shape[-1] // P
    taps = encoder_taps(w, cfg, x)
    if keep is not None:
        keep["taps"] = taps
    return dpt_head(w, cfg, taps, ph, pw, keep)

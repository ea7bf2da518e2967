"""ORACLE -- test infrastructure only.  CPU fp32 restatement of the VGGT
depth path: DINOv2-L/14 patch embedding with 4 registers, the alternating
frame / global attention aggregator (per-head q/k LayerNorm, 2D RoPE) and the
DPT depth head with its UV sin/cos positional embeddings.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker / the reported CPU baseline.  The
product path (`monocular_depth_estimation_trt_amd`) never calls it.

What it restates.  The reference exports facebookresearch/vggt's VGGT as
`VGGTDepthOnlyWrapper` (`models/vggt/onnx_export.py:38-52`: aggregator ->
depth_head, output "depth" only) under two export patches it ships itself:
`core/export_compat.py:84-93` (RoPE grid positions without cartesian_prod,
identical values) and `core/export_compat.py:145-152` (the UV embedding's
frequencies in float32 -- what the TensorRT engine computes).  The upstream
repository is cloned at run time and not vendored (`models/vggt/README.md`),
so the module arithmetic below is restated from upstream VGGT-1B
(`UP:` = vggt/ paths) and cross-checked where something executable exists:

* images / ImageNet mean-std, B*S frames              -- UP models/aggregator.py forward
* DINOv2 ViT-L/14-reg: conv patch embed, cls + pos, 4 registers after cls,
  pre-LN blocks (eps 1e-6) + LayerScale, final norm, patch tokens only
                                                        -- UP layers/vision_transformer.py
* camera + register tokens: set 0 for frame 0, set 1 for the others
                                                        -- UP aggregator.slice_expand_and_flatten
* RoPE positions: patch grid (y, x) + 1, special tokens (0, 0)
                                                        -- UP layers/rope.py PositionGetter,
                                                           reference export_compat.py:84-93
* 2D RoPE (base 100): first half of the head dim rotated by y, second by x,
  rotate_half within each half                          -- UP layers/rope.py RotaryPositionEmbedding2D
* blocks: LN(eps 1e-5) -> qkv -> q/k LayerNorm(64) -> RoPE -> SDPA -> proj,
  LayerScale; LN -> fc1 -> GELU -> fc2, LayerScale     -- UP layers/block.py, layers/attention.py
* frame blocks over [B*S, T], global blocks over [B, S*T]; intermediate i =
  cat(frame_out_i, global_out_i)                        -- UP aggregator._process_*_attention
* DPT head: LN(2048) on patch tokens of layers [4,11,17,23], 1x1 projects,
  + 0.1 * UV embed, resize (ConvT4 / ConvT2 / id / conv s2), layerN_rn,
  fusion blocks with in-place-ReLU residual units (the skip adds relu(x)),
  bilinear align_corners, output_conv1, upsample to the input size,
  + 0.1 * UV embed, output_conv2 (conv3 + ReLU + 1x1 -> 2), depth = exp(ch 0)
                                                        -- UP heads/dpt_head.py, heads/utils.py,
                                                           heads/head_act.py ("exp")

The token layout matches the reference's own description of the split export
(`models/vggt/onnx_export_split.py:49-59`: 24 x [B, S, 1374, 2048],
patch_start_idx 5 at 518^2) and the layer names of its TensorRT profile
(`reports/profile/vggt.json`).

Parity status: PARTIALLY PINNED.  The DINOv2-with-registers encoder is pinned
against transformers' `Dinov2WithRegistersModel` and the RoPE positions and
UV sin/cos tables against the reference's own `core/export_compat.py`
functions (tests/golden/make_golden_vggt.py -> tests/golden/vggt_*.npz).  The
aggregator blocks and the DPT head have no executable reference here (no
VGGT in transformers, upstream not vendored, no published vectors:
SURVEY.md 8c) -- they are unpinned restatements.
"""

from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

__all__ = ["forward", "to_torch", "aggregator", "depth_head", "dinov2_reg", "position_grid", "rope_positions",
           "rope2d", "rope_tables", "make_sincos_pos_embed", "create_uv_grid", "uv_embed"]

NUM_REG = 4
RESNET_MEAN = (0.485, 0.456, 0.406)
RESNET_STD = (0.229, 0.224, 0.225)


def to_torch(sd: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    return {k: torch.from_numpy(np.ascontiguousarray(v)).float() for k, v in sd.items()}


# ---- positions ------------------------------------------------------------
def position_grid(h: int, w: int) -> torch.Tensor:
    """UP PositionGetter: cartesian_prod(arange(h), arange(w)) -> [h*w, 2] (y, x),
    row-major (the reference's export patch builds the same values,
    export_compat.py:86-91)."""
    return torch.cartesian_prod(torch.arange(h), torch.arange(w))


def rope_positions(h: int, w: int, npre: int) -> torch.Tensor:
    """Per-frame token positions: special tokens (0, 0), patches grid + 1."""
    return torch.cat([torch.zeros(npre, 2, dtype=torch.long), position_grid(h, w) + 1], 0)


def rope_tables(dim: int, max_pos: int, base: float = 100.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """UP RotaryPositionEmbedding2D._compute_frequency_components(dim, max_pos):
    inv_freq = base^-(2j/dim), angles duplicated -> cos/sin [max_pos, dim] fp32."""
    exps = torch.arange(0, dim, 2).float() / dim
    inv = 1.0 / (base ** exps)
    ang = torch.einsum("i,j->ij", torch.arange(max_pos, dtype=inv.dtype), inv)
    ang = torch.cat((ang, ang), -1)
    return ang.cos(), ang.sin()


def _rope1d(x: torch.Tensor, p: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    c, s = cos[p], sin[p]                       # [T, d]
    h = x.shape[-1] // 2
    rot = torch.cat((-x[..., h:], x[..., :h]), -1)
    return x * c + rot * s


def rope2d(x: torch.Tensor, pos: torch.Tensor, base: float = 100.0) -> torch.Tensor:
    """x [..., T, dh]; pos [T, 2] (y, x).  First dh/2 features by y, rest by x."""
    d = x.shape[-1] // 2
    cos, sin = rope_tables(d, int(pos.max()) + 1, base)
    v, hz = x.chunk(2, -1)
    return torch.cat((_rope1d(v, pos[:, 0], cos, sin), _rope1d(hz, pos[:, 1], cos, sin)), -1)


# ---- UV sin/cos embedding of the DPT head --------------------------------
def make_sincos_pos_embed(embed_dim: int, pos: torch.Tensor, omega_0: float = 100.0,
                          float64: bool = False) -> torch.Tensor:
    """UP heads/utils.make_sincos_pos_embed.  float64=False is the reference
    export's float32 version (core/export_compat.py:145-152), the arithmetic
    of its engine; float64=True is upstream's eager double-precision path."""
    dt = torch.float64 if float64 else torch.float32
    omega = torch.arange(embed_dim // 2, dtype=dt)
    omega /= embed_dim / 2.0
    omega = 1.0 / omega_0 ** omega
    out = torch.einsum("m,d->md", pos.reshape(-1).to(dt), omega)
    return torch.cat([torch.sin(out), torch.cos(out)], 1).float()


def create_uv_grid(width: int, height: int, aspect_ratio: Optional[float] = None) -> torch.Tensor:
    """UP heads/utils.create_uv_grid -> [height, width, 2] (u, v) fp32."""
    if aspect_ratio is None:
        aspect_ratio = float(width) / float(height)
    diag = (aspect_ratio ** 2 + 1.0) ** 0.5
    span_x, span_y = aspect_ratio / diag, 1.0 / diag
    lx, rx = -span_x * (width - 1) / width, span_x * (width - 1) / width
    ty, by = -span_y * (height - 1) / height, span_y * (height - 1) / height
    xs = torch.linspace(lx, rx, steps=width, dtype=torch.float32)
    ys = torch.linspace(ty, by, steps=height, dtype=torch.float32)
    uu, vv = torch.meshgrid(xs, ys, indexing="xy")
    return torch.stack((uu, vv), -1)


def uv_embed(channels: int, h: int, w: int, aspect: float, ratio: float = 0.1, omega_0: float = 100.0,
             float64: bool = False) -> torch.Tensor:
    """UP DPTHead._apply_pos_embed's additive term -> [channels, h, w]:
    position_grid_to_embed(create_uv_grid(w, h, W/H), C) * ratio."""
    g = create_uv_grid(w, h, aspect).reshape(-1, 2)
    ex = make_sincos_pos_embed(channels // 2, g[:, 0], omega_0, float64)
    ey = make_sincos_pos_embed(channels // 2, g[:, 1], omega_0, float64)
    return (torch.cat([ex, ey], -1) * ratio).reshape(h, w, channels).permute(2, 0, 1)


# ---- transformer ----------------------------------------------------------
def _block(w, b: str, x: torch.Tensor, nh: int, eps: float, qk_norm: bool,
           pos: Optional[torch.Tensor] = None, rope_base: float = 100.0) -> torch.Tensor:
    """UP layers/block.py Block (+ layers/attention.py Attention)."""
    N, T, D = x.shape
    dh = D // nh
    h = F.layer_norm(x, (D,), w[b + "norm1.weight"], w[b + "norm1.bias"], eps)
    qkv = F.linear(h, w[b + "attn.qkv.weight"], w[b + "attn.qkv.bias"]).reshape(N, T, 3, nh, dh).permute(2, 0, 3, 1, 4)
    q, k, v = qkv.unbind(0)
    if qk_norm:
        q = F.layer_norm(q, (dh,), w[b + "attn.q_norm.weight"], w[b + "attn.q_norm.bias"], eps)
        k = F.layer_norm(k, (dh,), w[b + "attn.k_norm.weight"], w[b + "attn.k_norm.bias"], eps)
    if pos is not None:
        q = rope2d(q, pos, rope_base)
        k = rope2d(k, pos, rope_base)
    att = ((q @ k.transpose(-2, -1)) * dh ** -0.5).softmax(-1)
    o = (att @ v).transpose(1, 2).reshape(N, T, D)
    x = x + w[b + "ls1.gamma"] * F.linear(o, w[b + "attn.proj.weight"], w[b + "attn.proj.bias"])
    h = F.layer_norm(x, (D,), w[b + "norm2.weight"], w[b + "norm2.bias"], eps)
    h = F.linear(F.gelu(F.linear(h, w[b + "mlp.fc1.weight"], w[b + "mlp.fc1.bias"])),
                 w[b + "mlp.fc2.weight"], w[b + "mlp.fc2.bias"])
    return x + w[b + "ls2.gamma"] * h


def dinov2_reg(w, cfg: dict, x: torch.Tensor) -> torch.Tensor:
    """UP DinoVisionTransformer.forward_features(x)["x_norm_patchtokens"]:
    x normalised [N, 3, H, W] at the checkpoint's own grid -> [N, G*G, D]."""
    D, nh, P = cfg["embed_dim"], cfg["num_heads"], cfg["patch"]
    p = "aggregator.patch_embed."
    N = x.shape[0]
    t = F.conv2d(x, w[p + "patch_embed.proj.weight"], w[p + "patch_embed.proj.bias"], stride=P)
    t = t.flatten(2).transpose(1, 2)
    pos = w[p + "pos_embed"]
    if pos.shape[1] != t.shape[1] + 1:
        raise ValueError("the oracle runs VGGT at its checkpoint grid only (no pos-embed interpolation)")
    t = torch.cat([w[p + "cls_token"].expand(N, -1, -1), t], 1) + pos
    t = torch.cat([t[:, :1], w[p + "register_tokens"].expand(N, -1, -1), t[:, 1:]], 1)
    for i in range(cfg["depth"]):
        t = _block(w, f"{p}blocks.{i}.", t, nh, cfg["ln_eps"], False)
    t = F.layer_norm(t, (D,), w[p + "norm.weight"], w[p + "norm.bias"], cfg["ln_eps"])
    return t[:, 1 + NUM_REG:]


def _special(tok: torch.Tensor, B: int, S: int) -> torch.Tensor:
    """UP slice_expand_and_flatten: (1, 2, X, C) -> [B*S, X, C], set 0 for frame 0."""
    first = tok[:, 0:1].expand(B, 1, -1, -1)
    rest = tok[:, 1:].expand(B, S - 1, -1, -1)
    return torch.cat([first, rest], 1).reshape(B * S, tok.shape[2], tok.shape[3])


def aggregator(w, cfg: dict, images: torch.Tensor, keep_layers: Optional[Sequence[int]] = None
               ) -> Tuple[Dict[int, torch.Tensor], int, int]:
    """UP Aggregator.forward: images [B, S, 3, H, W] in [0, 1] ->
    ({layer: cat(frame_i, global_i) [B, S, T, 2D]}, T, patch_start_idx)."""
    B, S, _, H, W_ = images.shape
    D, nh, P = cfg["embed_dim"], cfg["num_heads"], cfg["patch"]
    eps, base = cfg["agg_eps"], cfg["rope_freq"]
    keep = set(cfg["taps"] if keep_layers is None else keep_layers)
    mean = torch.tensor(RESNET_MEAN).view(1, 1, 3, 1, 1)
    std = torch.tensor(RESNET_STD).view(1, 1, 3, 1, 1)
    x = ((images - mean) / std).reshape(B * S, 3, H, W_)
    pt = dinov2_reg(w, cfg, x)
    tok = torch.cat([_special(w["aggregator.camera_token"], B, S),
                     _special(w["aggregator.register_token"], B, S), pt], 1)
    npre = 1 + NUM_REG
    T = tok.shape[1]
    pos = rope_positions(H // P, W_ // P, npre)
    pos_g = pos.repeat(S, 1)
    outs: Dict[int, torch.Tensor] = {}
    for i in range(cfg["aa_depth"]):
        tok = _block(w, f"aggregator.frame_blocks.{i}.", tok.reshape(B * S, T, D), nh, eps, True, pos, base)
        fr = tok.reshape(B, S, T, D)
        tok = _block(w, f"aggregator.global_blocks.{i}.", tok.reshape(B, S * T, D), nh, eps, True, pos_g, base)
        if i in keep:
            outs[i] = torch.cat([fr, tok.reshape(B, S, T, D)], -1)
    return outs, T, npre


# ---- DPT head -------------------------------------------------------------
def _rcu(w, pfx: str, x: torch.Tensor) -> torch.Tensor:
    """UP ResidualConvUnit with nn.ReLU(inplace=True): the first activation
    overwrites x, so the skip connection adds relu(x)."""
    xr = F.relu(x)
    o = F.conv2d(xr, w[pfx + "conv1.weight"], w[pfx + "conv1.bias"], padding=1)
    o = F.conv2d(F.relu(o), w[pfx + "conv2.weight"], w[pfx + "conv2.bias"], padding=1)
    return o + xr


def _fusion(w, pfx: str, x0: torch.Tensor, x1: Optional[torch.Tensor], size=None) -> torch.Tensor:
    """UP FeatureFusionBlock (align_corners=True, has_residual = x1 given)."""
    out = x0
    if x1 is not None:
        out = out + _rcu(w, pfx + "resConfUnit1.", x1)
    out = _rcu(w, pfx + "resConfUnit2.", out)
    if size is None:
        out = F.interpolate(out, scale_factor=2, mode="bilinear", align_corners=True)
    else:
        out = F.interpolate(out, size=size, mode="bilinear", align_corners=True)
    return F.conv2d(out, w[pfx + "out_conv.weight"], w[pfx + "out_conv.bias"])


def depth_head(w, cfg: dict, outs: Dict[int, torch.Tensor], H: int, W_: int, npre: int,
               keep: Optional[dict] = None) -> torch.Tensor:
    """UP DPTHead._forward_impl (+ activate_head "exp") -> depth [B, S, H, W, 1]."""
    h = "depth_head."
    P = cfg["patch"]
    ph, pw = H // P, W_ // P
    aspect = float(W_) / float(H)
    r = cfg["pe_ratio"]
    feats = []
    for k, li in enumerate(cfg["taps"]):
        t = outs[li]
        B, S = t.shape[:2]
        x = t[:, :, npre:].reshape(B * S, ph * pw, t.shape[-1])
        x = F.layer_norm(x, (t.shape[-1],), w[h + "norm.weight"], w[h + "norm.bias"], cfg["agg_eps"])
        x = x.permute(0, 2, 1).reshape(B * S, -1, ph, pw)
        x = F.conv2d(x, w[f"{h}projects.{k}.weight"], w[f"{h}projects.{k}.bias"])
        x = x + uv_embed(x.shape[1], ph, pw, aspect, r)
        if k == 0:
            x = F.conv_transpose2d(x, w[h + "resize_layers.0.weight"], w[h + "resize_layers.0.bias"], stride=4)
        elif k == 1:
            x = F.conv_transpose2d(x, w[h + "resize_layers.1.weight"], w[h + "resize_layers.1.bias"], stride=2)
        elif k == 3:
            x = F.conv2d(x, w[h + "resize_layers.3.weight"], w[h + "resize_layers.3.bias"], stride=2, padding=1)
        feats.append(x)
    s = h + "scratch."
    l = [F.conv2d(f, w[f"{s}layer{i + 1}_rn.weight"], padding=1) for i, f in enumerate(feats)]
    out = _fusion(w, s + "refinenet4.", l[3], None, l[2].shape[2:])
    out = _fusion(w, s + "refinenet3.", out, l[2], l[1].shape[2:])
    out = _fusion(w, s + "refinenet2.", out, l[1], l[0].shape[2:])
    out = _fusion(w, s + "refinenet1.", out, l[0], None)
    out = F.conv2d(out, w[s + "output_conv1.weight"], w[s + "output_conv1.bias"], padding=1)
    out = F.interpolate(out, size=(ph * P, pw * P), mode="bilinear", align_corners=True)
    out = out + uv_embed(out.shape[1], ph * P, pw * P, aspect, r)
    out = F.relu(F.conv2d(out, w[s + "output_conv2.0.weight"], w[s + "output_conv2.0.bias"], padding=1))
    out = F.conv2d(out, w[s + "output_conv2.2.weight"], w[s + "output_conv2.2.bias"])
    if keep is not None:
        keep.update(feats=feats, rn=l, head_logits=out)
    B, S = outs[cfg["taps"][0]].shape[:2]
    return torch.exp(out[:, 0]).reshape(B, S, ph * P, pw * P, 1)


@torch.no_grad()
def forward(w: Dict[str, torch.Tensor], cfg: dict, images, keep: Optional[dict] = None) -> torch.Tensor:
    """VGGTDepthOnlyWrapper.forward (reference onnx_export.py:42-52):
    images float32 [B, S, 3, H, W] in [0, 1] -> depth [B, S, H, W, 1]."""
    if isinstance(images, np.ndarray):
        images = torch.from_numpy(images)
    images = images.float()
    if images.ndim == 4:
        images = images[None]
    H, W_ = images.shape[-2:]
    outs, _, npre = aggregator(w, cfg, images)
    if keep is not None:
        keep["tokens"] = outs
    return depth_head(w, cfg, outs, H, W_, npre, keep)

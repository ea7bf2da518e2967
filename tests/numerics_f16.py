"""Test helper (not a test module): the DA-V2 oracle forward with fp16
STORAGE emulated at chosen stages -- the same fp32 arithmetic as
oracle/dav2_ref.py (whose pieces it reuses), with `.half().float()` applied
where the fp16 engine stores a tensor in fp16.  Used to attribute the fp16
engine's worst pixels to the stage whose fp16 rounding
the output amplifies.

Stages (the engine's f16 storage points):
  resid  -- the residual stream after the patch embed and every residual update
  enc    -- the encoder's GEMM inputs / outputs: LN output, q, k, v, softmax
            probabilities, attention output, MLP hidden (f16 operands)
  taps   -- the normed tap token maps the DPT projects read
  dpt    -- every DPT map (projects, resize layers, layerN_rn, RCU
            intermediates, fusion outputs)
  head   -- output_conv1's output and its bilinear upsample to full size
  w16    -- every weight matrix / kernel (>= 2-D) rounded to fp16, as packed
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle import dav2_ref as R

STAGES = ("resid", "enc", "taps", "dpt", "head", "w16")


def _q(on):
    return (lambda x: x.half().float()) if on else (lambda x: x)


def encoder_taps(w, cfg, x, stages):
    qr, qe = _q("resid" in stages), _q("enc" in stages)
    B, _, H, W = x.shape
    P = cfg["patch"]
    ph, pw = H // P, W // P
    D, nh = cfg["embed_dim"], cfg["num_heads"]
    dh = D // nh
    eps = cfg["ln_eps"]
    p = "pretrained."
    t = F.conv2d(x, w[p + "patch_embed.proj.weight"], w[p + "patch_embed.proj.bias"], stride=P)
    t = t.flatten(2).transpose(1, 2)
    t = torch.cat([w[p + "cls_token"].expand(B, -1, -1), t], dim=1)
    t = qr(t + R.interpolate_pos_embed(w[p + "pos_embed"], ph, pw))
    T = t.shape[1]
    taps = []
    for i in range(cfg["depth"]):
        b = f"{p}blocks.{i}."
        h = qe(F.layer_norm(t, (D,), w[b + "norm1.weight"], w[b + "norm1.bias"], eps))
        qkv = F.linear(h, w[b + "attn.qkv.weight"], w[b + "attn.qkv.bias"])
        qkv = qkv.reshape(B, T, 3, nh, dh).permute(2, 0, 3, 1, 4)
        q, k, v = qe(qkv[0] * (dh ** -0.5)), qe(qkv[1]), qe(qkv[2])
        a = qe((q @ k.transpose(-2, -1)).softmax(dim=-1))
        o = qe((a @ v).transpose(1, 2).reshape(B, T, D))
        o = F.linear(o, w[b + "attn.proj.weight"], w[b + "attn.proj.bias"])
        t = qr(t + w[b + "ls1.gamma"] * o)
        h = qe(F.layer_norm(t, (D,), w[b + "norm2.weight"], w[b + "norm2.bias"], eps))
        h = qe(F.gelu(F.linear(h, w[b + "mlp.fc1.weight"], w[b + "mlp.fc1.bias"])))
        h = F.linear(h, w[b + "mlp.fc2.weight"], w[b + "mlp.fc2.bias"])
        t = qr(t + w[b + "ls2.gamma"] * h)
        if i in cfg["taps"]:
            taps.append(F.layer_norm(t, (D,), w[p + "norm.weight"], w[p + "norm.bias"], eps))
    return taps


def _rcu(w, pre, x, q):
    o = F.relu(x)
    o = q(F.conv2d(o, w[pre + "conv1.weight"], w[pre + "conv1.bias"], padding=1))
    o = F.relu(o)
    o = F.conv2d(o, w[pre + "conv2.weight"], w[pre + "conv2.bias"], padding=1)
    return q(o + x)


def _fusion(w, pre, x0, x1, size, q):
    out = x0
    if x1 is not None:
        out = q(out + _rcu(w, pre + "resConfUnit1.", x1, q))
    out = _rcu(w, pre + "resConfUnit2.", out, q)
    if size is None:
        size = (out.shape[2] * 2, out.shape[3] * 2)
    # the engine applies out_conv (1x1) before the resize (exact in real
    # arithmetic) and stores the resized map in f16
    out = F.conv2d(out, w[pre + "out_conv.weight"], w[pre + "out_conv.bias"])
    return q(R.bilinear_ac(out, size))


def dpt_head(w, cfg, taps, ph, pw, stages):
    qt, qd, qh = _q("taps" in stages), _q("dpt" in stages), _q("head" in stages)
    h = "depth_head."
    B = taps[0].shape[0]
    feats = []
    for i, t in enumerate(taps):
        t = qt(t[:, 1:])
        t = t.permute(0, 2, 1).reshape(B, t.shape[-1], ph, pw)
        t = qd(F.conv2d(t, w[f"{h}projects.{i}.weight"], w[f"{h}projects.{i}.bias"]))
        if i == 0:
            t = F.conv_transpose2d(t, w[h + "resize_layers.0.weight"], w[h + "resize_layers.0.bias"], stride=4)
        elif i == 1:
            t = F.conv_transpose2d(t, w[h + "resize_layers.1.weight"], w[h + "resize_layers.1.bias"], stride=2)
        elif i == 3:
            t = F.conv2d(t, w[h + "resize_layers.3.weight"], w[h + "resize_layers.3.bias"], stride=2, padding=1)
        feats.append(qd(t))
    rn = [qd(F.conv2d(f, w[f"{h}scratch.layer{i + 1}_rn.weight"], None, padding=1)) for i, f in enumerate(feats)]
    s = h + "scratch."
    p4 = _fusion(w, s + "refinenet4.", rn[3], None, rn[2].shape[2:], qd)
    p3 = _fusion(w, s + "refinenet3.", p4, rn[2], rn[1].shape[2:], qd)
    p2 = _fusion(w, s + "refinenet2.", p3, rn[1], rn[0].shape[2:], qd)
    p1 = _fusion(w, s + "refinenet1.", p2, rn[0], None, qd)
    o = qh(F.conv2d(p1, w[s + "output_conv1.weight"], w[s + "output_conv1.bias"], padding=1))
    o = qh(R.bilinear_ac(o, (ph * cfg["patch"], pw * cfg["patch"])))
    o = F.conv2d(o, w[s + "output_conv2.0.weight"], w[s + "output_conv2.0.bias"], padding=1)
    o = F.relu(o)
    o = F.conv2d(o, w[s + "output_conv2.2.weight"], w[s + "output_conv2.2.bias"])
    pre = o.squeeze(1)
    if cfg["depth_type"] == "metric":
        o = torch.sigmoid(o) * cfg["max_depth"]
    else:
        o = F.relu(o)
    return o.squeeze(1), pre


@torch.no_grad()
def forward(w, cfg, x, stages=()):
    """-> (depth [B, H, W], the pre-activation logit map [B, H, W])."""
    if not isinstance(x, torch.Tensor):
        x = torch.from_numpy(x)
    x = x.float()
    if "w16" in stages:
        w = {k: (v.half().float() if v.dim() >= 2 else v) for k, v in w.items()}
    P = cfg["patch"]
    ph, pw = x.shape[-2] // P, x.shape[-1] // P
    taps = encoder_taps(w, cfg, x, set(stages))
    return dpt_head(w, cfg, taps, ph, pw, set(stages))

"""AOT weight packer: DA-V2 state dict -> packed engine file for libmde_hip.

Replaces the reference's export/build stage -- `run.py export` ->
`models/depth_anything_v2/onnx_export.py:19-100` (ONNX opset 20 + onnxsim)
and `run.py build` -> `core/common.py:166-274` (TensorRT builder) -- with one
deterministic host-side pass that lays the weights out for the gfx950 kernels:

* every matrix operand becomes f16 [Npad][Kpad] (K contiguous; N padded to a
  multiple of 128 and K to a multiple of 64 with zeros) -- the B-operand
  layout of the MFMA GEMM (csrc/gemm.hip);
* 3x3 conv weights [Cout][Cin][3][3] -> [Cout][ky][kx][Cin] (the implicit
  im2col K order over an NHWC map);
* ConvTranspose(k == s) weights [Cin][Cout][s][s] -> [(dy*s+dx)*Cout+co][Cin]
  (a plain GEMM whose epilogue pixel-shuffles);
* patch-embed [D][3][14][14] -> [D][3*14*16] (kx padded to 16 so every 8-wide
  K chunk of the im2col row is 16-byte aligned);
* the positional table is interpolated ONCE for the packed input size with
  upstream DINOv2's bicubic + 0.1-offset rule, and cls + pos[0] is folded;
* LayerNorm / LayerScale / bias vectors stay fp32.

File layout: csrc/pack_format.h.  A packed file is specific to one model
variant and one input size, like a TensorRT engine is to its profile.
"""

from __future__ import annotations

import hashlib
import math
import os
import struct
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

from . import weights as W

PACK_VERSION = 1
PACKER_VERSION = "mde-pack-1"
ALIGN = 256


def _pad2(a: np.ndarray, n_mult: int = 128, k_mult: int = 64) -> np.ndarray:
    n, k = a.shape
    N = -(-n // n_mult) * n_mult
    K = -(-k // k_mult) * k_mult
    out = np.zeros((N, K), np.float16)
    out[:n, :k] = a.astype(np.float16)
    return out


def _pad2_f32(a: np.ndarray, n_mult: int = 128, k_mult: int = 32) -> np.ndarray:
    """fp32 [Npad][Kpad] (N -> x128, K -> x32, zero padded): the exact-fp32
    GEMM's weight operand (csrc/fp32.hip)."""
    n, k = a.shape
    out = np.zeros((-(-n // n_mult) * n_mult, -(-k // k_mult) * k_mult), np.float32)
    out[:n, :k] = np.asarray(a, np.float32)
    return out


def _conv3(w: np.ndarray, cin_pad: int = 0) -> np.ndarray:
    """[Cout][Cin][3][3] -> f16 [Cout_pad][9*Cin' pad64] in (ky, kx, ci) order,
    Cin' = cin_pad (zero input channels appended) when given."""
    co, ci, kh, kw = w.shape
    assert kh == 3 and kw == 3, w.shape
    if cin_pad and cin_pad > ci:
        w = np.concatenate([w, np.zeros((co, cin_pad - ci, 3, 3), w.dtype)], axis=1)
        ci = cin_pad
    return _pad2(np.ascontiguousarray(w.transpose(0, 2, 3, 1)).reshape(co, 9 * ci))


def _convT(w: np.ndarray) -> np.ndarray:
    """ConvTranspose2d weight [Cin][Cout][s][s] (k == s) -> [(dy*s+dx)*Cout+co][Cin]."""
    ci, co, s, s2 = w.shape
    assert s == s2
    return _pad2(np.ascontiguousarray(w.transpose(2, 3, 1, 0)).reshape(s * s * co, ci))


def _conv3_f32(w: np.ndarray) -> np.ndarray:
    """[Cout][Cin][3][3] -> fp32 [Cout_pad][9*Cin pad32] in (ky, kx, ci) order:
    the exact-fp32 implicit-im2col conv's weight operand (csrc/fp32.hip)."""
    co, ci, kh, kw = w.shape
    assert kh == 3 and kw == 3, w.shape
    return _pad2_f32(np.ascontiguousarray(w.transpose(0, 2, 3, 1)).reshape(co, 9 * ci))


def _convT_f32(w: np.ndarray) -> np.ndarray:
    """ConvTranspose2d weight [Cin][Cout][s][s] (k == s) -> fp32 [(dy*s+dx)*Cout+co][Cin]."""
    ci, co, s, s2 = w.shape
    assert s == s2
    return _pad2_f32(np.ascontiguousarray(w.transpose(2, 3, 1, 0)).reshape(s * s * co, ci))


def interpolate_pos_embed(pos: np.ndarray, ph: int, pw: int) -> np.ndarray:
    """Upstream DINOv2 interpolate_pos_encoding (bicubic, scale_factor with the
    0.1 offset, antialias False).  [1, 1+M*M, D] -> [1, 1+ph*pw, D] fp32."""
    N = pos.shape[1] - 1
    if N == ph * pw and ph == pw:
        return pos.astype(np.float32)
    import torch
    import torch.nn.functional as F
    M = int(math.isqrt(N))
    if M * M != N:
        raise ValueError(f"pos_embed has {N} patch positions, not a square grid")
    D = pos.shape[-1]
    t = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.float32))
    patch = t[:, 1:].reshape(1, M, M, D).permute(0, 3, 1, 2)
    patch = F.interpolate(patch, scale_factor=(float(ph + 0.1) / M, float(pw + 0.1) / M),
                          mode="bicubic", antialias=False)
    if tuple(patch.shape[-2:]) != (ph, pw):
        raise ValueError(f"pos-embed interpolation produced {tuple(patch.shape[-2:])}, wanted {(ph, pw)}")
    patch = patch.permute(0, 2, 3, 1).reshape(1, ph * pw, D)
    return torch.cat([t[:, :1], patch], 1).numpy()


def normalize_keys(sd: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Accept upstream checkpoints as saved (optionally 'module.'-prefixed)."""
    out = {}
    for k, v in sd.items():
        if k.startswith("module."):
            k = k[len("module."):]
        out[k] = np.asarray(v.detach().cpu().numpy() if hasattr(v, "detach") else v, dtype=np.float32)
    return out


def _fold_ln(w: np.ndarray, bias: np.ndarray, g: np.ndarray, beta: np.ndarray):
    """LayerNorm folded into the linear that follows it (the f16-residual
    engines' norm1 -> qkv and norm2 -> fc1, engine.hip): with x the raw
    residual row, LN(x) W^T + b = rstd * (x (W*g)^T - mean * c1) + c2, where
    W*g scales input column k by gamma[k], c1[n] = sum_k f16(W*g)[n][k] (the
    operand the MFMAs see) and c2 = b + f16(W) beta.  Returns the padded f16
    W*g, c1 and c2 (fp32, sums in fp64)."""
    w = np.asarray(w, np.float32)
    wg = (w.astype(np.float64) * np.asarray(g, np.float64)[None, :]).astype(np.float32)
    c1 = wg.astype(np.float16).astype(np.float64).sum(axis=1)
    c2 = np.asarray(bias, np.float64) + w.astype(np.float16).astype(np.float64) @ np.asarray(beta, np.float64)
    return _pad2(wg), c1.astype(np.float32), c2.astype(np.float32)


def _slice_partials(v: np.ndarray) -> np.ndarray:
    """Per 32-column slice, (sum, sum of squared deviations from the slice
    mean) of the f16-rounded row v -- the LayerNorm partials the fold's
    producers write (GemmParams::lnst_out)."""
    h = np.asarray(v, np.float32).astype(np.float16).astype(np.float64).reshape(-1, 32)
    m2 = ((h - h.mean(1, keepdims=True)) ** 2).sum(1)
    return np.stack([h.sum(1), m2], 1).astype(np.float32).reshape(-1)


def packed_tensors(sd: Dict[str, np.ndarray], cfg: dict, img_h: int, img_w: int,
                   fold_ln: bool = False, enc_f32: bool = False) -> "OrderedDict[str, np.ndarray]":
    """The packed tensors (name -> f16/f32 numpy array) for one input size.
    fold_ln (precision "fp16" engines) adds the LayerNorm-folded qkv / fc1 /
    DPT project weights (`*.wf`, `*.c1`, `*.c2`) and the cls row's partials
    (`pos.cls.st`).  enc_f32 (precision "fp32" engines) stores the patch
    embed and the block linears as fp32 (`*.w32`) in place of f16."""
    sd = normalize_keys(sd)
    missing = [k for k in W.expected_keys(cfg) if k not in sd and not k.endswith("mask_token")]
    if missing:
        raise KeyError(f"state dict lacks {len(missing)} keys, e.g. {missing[:4]}")
    P = cfg["patch"]
    if img_h % P or img_w % P:
        raise ValueError(f"input size {img_h}x{img_w} is not a multiple of the patch size {P}")
    ph, pw = img_h // P, img_w // P
    D = cfg["embed_dim"]
    f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1)  # noqa: E731
    o: "OrderedDict[str, np.ndarray]" = OrderedDict()
    p = "pretrained."
    pe = sd[p + "patch_embed.proj.weight"]                   # [D,3,14,14]
    pe16 = np.zeros((D, 3, 14, 16), np.float32)
    pe16[..., :14] = pe
    if enc_f32:
        o["patch.w32"] = _pad2_f32(pe16.reshape(D, 3 * 14 * 16))
    else:
        o["patch.w"] = _pad2(pe16.reshape(D, 3 * 14 * 16))
    o["patch.b"] = f32(sd[p + "patch_embed.proj.bias"])
    pos = interpolate_pos_embed(sd[p + "pos_embed"], ph, pw)
    o["pos.patch"] = np.ascontiguousarray(pos[0, 1:], dtype=np.float32)
    o["pos.cls"] = f32(sd[p + "cls_token"].reshape(-1) + pos[0, 0])
    if fold_ln and D % 32 == 0:
        o["pos.cls.st"] = _slice_partials(o["pos.cls"])
    for i in range(cfg["depth"]):
        b = f"{p}blocks.{i}."
        q = f"b{i}."
        o[q + "ln1.g"] = f32(sd[b + "norm1.weight"])
        o[q + "ln1.b"] = f32(sd[b + "norm1.bias"])
        lin = (lambda a: _pad2_f32(a)) if enc_f32 else _pad2  # noqa: E731
        wsuf = ".w32" if enc_f32 else ".w"
        o[q + "qkv" + wsuf] = lin(sd[b + "attn.qkv.weight"])
        o[q + "qkv.b"] = f32(sd[b + "attn.qkv.bias"])
        o[q + "proj" + wsuf] = lin(sd[b + "attn.proj.weight"])
        o[q + "proj.b"] = f32(sd[b + "attn.proj.bias"])
        o[q + "ls1"] = f32(sd[b + "ls1.gamma"])
        o[q + "ln2.g"] = f32(sd[b + "norm2.weight"])
        o[q + "ln2.b"] = f32(sd[b + "norm2.bias"])
        o[q + "fc1" + wsuf] = lin(sd[b + "mlp.fc1.weight"])
        o[q + "fc1.b"] = f32(sd[b + "mlp.fc1.bias"])
        if fold_ln:
            o[q + "qkv.wf"], o[q + "qkv.c1"], o[q + "qkv.c2"] = _fold_ln(
                sd[b + "attn.qkv.weight"], sd[b + "attn.qkv.bias"], sd[b + "norm1.weight"], sd[b + "norm1.bias"])
            o[q + "fc1.wf"], o[q + "fc1.c1"], o[q + "fc1.c2"] = _fold_ln(
                sd[b + "mlp.fc1.weight"], sd[b + "mlp.fc1.bias"], sd[b + "norm2.weight"], sd[b + "norm2.bias"])
        o[q + "fc2" + wsuf] = lin(sd[b + "mlp.fc2.weight"])
        o[q + "fc2.b"] = f32(sd[b + "mlp.fc2.bias"])
        o[q + "ls2"] = f32(sd[b + "ls2.gamma"])
    o["norm.g"] = f32(sd[p + "norm.weight"])
    o["norm.b"] = f32(sd[p + "norm.bias"])
    h = "depth_head."
    if enc_f32:
        # the exact-fp32 engine's DPT head: every conv / linear weight fp32
        # (`*.w32`), the head run on fp32 maps (engine.hip dav2_head32)
        _head_f32(sd, cfg, o, f32)
        return o
    for i in range(4):
        w = sd[f"{h}projects.{i}.weight"]
        o[f"proj{i}.w"] = _pad2(w.reshape(w.shape[0], w.shape[1]))
        o[f"proj{i}.b"] = f32(sd[f"{h}projects.{i}.bias"])
        if fold_ln:  # the taps' final LayerNorm folded into the projects (engine.hip)
            o[f"proj{i}.wf"], o[f"proj{i}.c1"], o[f"proj{i}.c2"] = _fold_ln(
                w.reshape(w.shape[0], w.shape[1]), sd[f"{h}projects.{i}.bias"], sd[p + "norm.weight"],
                sd[p + "norm.bias"])
    o["rs0.w"] = _convT(sd[h + "resize_layers.0.weight"])
    o["rs0.b"] = f32(sd[h + "resize_layers.0.bias"])
    o["rs1.w"] = _convT(sd[h + "resize_layers.1.weight"])
    o["rs1.b"] = f32(sd[h + "resize_layers.1.bias"])
    o["rs3.w"] = _conv3(sd[h + "resize_layers.3.weight"])
    o["rs3.b"] = f32(sd[h + "resize_layers.3.bias"])
    for i in range(4):
        # DPT maps feeding the direct conv carry channels padded to x32 (48 -> 64)
        o[f"rn{i + 1}.w"] = _conv3(sd[f"{h}scratch.layer{i + 1}_rn.weight"], -(-cfg["out_channels"][i] // 32) * 32)
    for r in range(1, 5):
        s = f"{h}scratch.refinenet{r}."
        w = sd[s + "out_conv.weight"]
        o[f"rf{r}.out.w"] = _pad2(w.reshape(w.shape[0], w.shape[1]))
        o[f"rf{r}.out.b"] = f32(sd[s + "out_conv.bias"])
        for u in (1, 2):
            for c in (1, 2):
                o[f"rf{r}.rcu{u}.c{c}.w"] = _conv3(sd[f"{s}resConfUnit{u}.conv{c}.weight"])
                o[f"rf{r}.rcu{u}.c{c}.b"] = f32(sd[f"{s}resConfUnit{u}.conv{c}.bias"])
    s = h + "scratch."
    o["head.c1.w"] = _conv3(sd[s + "output_conv1.weight"])
    o["head.c1.b"] = f32(sd[s + "output_conv1.bias"])
    o["head.c2.w"] = _conv3(sd[s + "output_conv2.0.weight"])
    o["head.c2.b"] = f32(sd[s + "output_conv2.0.bias"])
    o["head.c3.w"] = f32(sd[s + "output_conv2.2.weight"])
    o["head.c3.b"] = f32(sd[s + "output_conv2.2.bias"])
    return o


def _head_f32(sd, cfg, o, f32) -> None:
    """fp32 DPT head weights: the f16 head's tensors under `.w32` names, no
    channel padding (the fp32 conv takes any channel count % 4)."""
    h = "depth_head."
    for i in range(4):
        w = sd[f"{h}projects.{i}.weight"]
        o[f"proj{i}.w32"] = _pad2_f32(w.reshape(w.shape[0], w.shape[1]))
        o[f"proj{i}.b"] = f32(sd[f"{h}projects.{i}.bias"])
    o["rs0.w32"] = _convT_f32(sd[h + "resize_layers.0.weight"])
    o["rs0.b"] = f32(sd[h + "resize_layers.0.bias"])
    o["rs1.w32"] = _convT_f32(sd[h + "resize_layers.1.weight"])
    o["rs1.b"] = f32(sd[h + "resize_layers.1.bias"])
    o["rs3.w32"] = _conv3_f32(sd[h + "resize_layers.3.weight"])
    o["rs3.b"] = f32(sd[h + "resize_layers.3.bias"])
    for i in range(4):
        o[f"rn{i + 1}.w32"] = _conv3_f32(sd[f"{h}scratch.layer{i + 1}_rn.weight"])
    for r in range(1, 5):
        s = f"{h}scratch.refinenet{r}."
        w = sd[s + "out_conv.weight"]
        o[f"rf{r}.out.w32"] = _pad2_f32(w.reshape(w.shape[0], w.shape[1]))
        o[f"rf{r}.out.b"] = f32(sd[s + "out_conv.bias"])
        for u in (1, 2):
            for c in (1, 2):
                o[f"rf{r}.rcu{u}.c{c}.w32"] = _conv3_f32(sd[f"{s}resConfUnit{u}.conv{c}.weight"])
                o[f"rf{r}.rcu{u}.c{c}.b"] = f32(sd[f"{s}resConfUnit{u}.conv{c}.bias"])
    s = h + "scratch."
    o["head.c1.w32"] = _conv3_f32(sd[s + "output_conv1.weight"])
    o["head.c1.b"] = f32(sd[s + "output_conv1.bias"])
    o["head.c2.w32"] = _conv3_f32(sd[s + "output_conv2.0.weight"])
    o["head.c2.b"] = f32(sd[s + "output_conv2.0.bias"])
    o["head.c3.w"] = f32(sd[s + "output_conv2.2.weight"])
    o["head.c3.b"] = f32(sd[s + "output_conv2.2.bias"])


INPUT_FORMATS = ("float32_nchw", "uint8_nhwc")
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


PRECISIONS = ("fp16", "fp32")


def _config_bytes(cfg: dict, img_h: int, img_w: int, input_format: str = "float32_nchw",
                  mean=IMAGENET_MEAN, std=IMAGENET_STD, scale: float = 255.0, precision: str = "fp16") -> bytes:
    """PackConfig (csrc/pack_format.h).  input_format "uint8_nhwc" stores the
    preamble constants of the reference's add_uint8_input
    (core/onnx_tools.py:87-219): ((u8 / scale) - mean) / std, fp32.
    precision "fp16" keeps the residual stream in f16 (resid_f16 = 1, the
    reference's fp16 TensorRT engine); "fp32" (the reference's default) runs
    the encoder exactly in fp32 (enc_f32 = 1: fp32 weights, activations and
    MFMA, csrc/fp32.hip)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}, got {precision!r}")
    if input_format not in INPUT_FORMATS:
        raise ValueError(f"input_format must be one of {INPUT_FORMATS}, got {input_format!r}")
    oc, taps = cfg["out_channels"], cfg["taps"]
    b = struct.pack("<8i4i4i2i2f16s", cfg["embed_dim"], cfg["depth"], cfg["num_heads"], cfg["mlp_hidden"],
                    cfg["patch"], img_h, img_w, cfg["features"], *oc, *taps, cfg["head_hidden"],
                    1 if cfg["depth_type"] == "metric" else 0, float(cfg["max_depth"]), float(cfg["ln_eps"]),
                    cfg["encoder"].encode()[:15])
    assert len(b) == 96, len(b)
    u8 = input_format == "uint8_nhwc"
    if u8 and (len(mean) != 3 or len(std) != 3 or float(scale) == 0.0 or any(float(v) == 0.0 for v in std)):
        raise ValueError("uint8 preamble needs 3 means, 3 non-zero stds and a non-zero scale")
    b += struct.pack("<if3f3f", 1 if u8 else 0, float(scale) if u8 else 0.0,
                     *([float(v) for v in mean] if u8 else [0.0] * 3),
                     *([float(v) for v in std] if u8 else [0.0] * 3))
    assert len(b) == 128, len(b)
    b += b"\0" * 68 + struct.pack("<i", 1 if precision == "fp16" else 0)   # resid_f16 at byte 196
    b += struct.pack("<i", 1 if precision == "fp32" else 0)                 # enc_f32 at byte 200
    return b + b"\0" * 52


def container(tens: "OrderedDict[str, np.ndarray]", cfg_bytes: bytes) -> bytes:
    """Header + PackConfig + tensor table + 256-byte aligned data."""
    assert len(cfg_bytes) == 256, len(cfg_bytes)
    n = len(tens)
    table = bytearray()
    data = bytearray()
    for name, a in tens.items():
        a = np.ascontiguousarray(a)
        dtype = {np.dtype(np.float32): 0, np.dtype(np.float16): 1}[a.dtype]
        if len(name) >= 80:
            raise ValueError(f"tensor name too long: {name}")
        dims = list(a.shape) + [0] * (4 - a.ndim)
        off = len(data)
        raw = a.tobytes()
        data += raw
        data += b"\0" * ((-len(data)) % ALIGN)
        table += struct.pack("<80sii4iQQ8s", name.encode(), dtype, a.ndim, *dims, off, len(raw), b"")
    head_len = 32 + 256 + len(table)
    data_offset = -(-head_len // ALIGN) * ALIGN
    header = struct.pack("<8sIIQQ", b"MDEPACK1", PACK_VERSION, n, data_offset, len(data))
    blob = header + cfg_bytes + bytes(table)
    blob += b"\0" * (data_offset - len(blob))
    return blob + bytes(data)


def pack_bytes(sd: Dict[str, np.ndarray], cfg: dict, img_h: int = 518, img_w: int = 518,
               input_format: str = "float32_nchw", precision: str = "fp16") -> bytes:
    return container(packed_tensors(sd, cfg, img_h, img_w, fold_ln=precision == "fp16", enc_f32=precision == "fp32"),
                     _config_bytes(cfg, img_h, img_w, input_format, precision=precision))


def write_packed(path: str, blob: bytes) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(blob)
    os.replace(tmp, path)
    return path


def synthetic_blob(encoder: str = "vits", depth_type: str = "metric", img_h: int = 518, img_w: int = 518,
                   seed: int = 1234, input_format: str = "float32_nchw") -> Tuple[bytes, dict]:
    cfg = W.model_config(encoder, depth_type)
    sd = W.synthetic_state_dict(cfg, seed)
    return pack_bytes(sd, cfg, img_h, img_w, input_format), cfg


def fingerprint(blob: bytes, arch: str = "gfx950") -> str:
    return "\n".join([hashlib.sha256(blob).hexdigest(), f"packer={PACKER_VERSION}", f"arch={arch}"])

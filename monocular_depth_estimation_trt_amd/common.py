"""get_engine(): build-or-load a packed engine -- the drop-in for the
reference's `core/common.py:141-312`.

The reference builds a TensorRT plan from an ONNX file (fingerprinted by
sha256 of the ONNX + builder options, :92-117; stale-engine detection,
:120-138) and deserializes it.  Here the "source" is a DA-V2 checkpoint (or a
`synthetic:` spec), the build step is the AOT weight packer (pack.py), and
the artefact is a packed engine file loaded by libmde_hip.  Same signature,
same reuse/rebuild rules, same errors (FileNotFoundError for a missing
source, RuntimeError for a failed build/load).

Source strings:
  synthetic:<vits|vitb|vitl>[:<metric|relative>[:<seed>]]   seeded DA-V2 weights
  synthetic:depth_pro[:<dinov2l16_384|tiny>[:<seed>]]       seeded Depth Pro weights
  synthetic:vggt[:<vggt_1b|vggt_1b_shallow|tiny>[:<seed>]]  seeded VGGT weights (depth path)
  /path/ckpt.pth          torch.load(..., weights_only=True)
  /path/ckpt.safetensors  safetensors
  /path/ckpt.npz          numpy (allow_pickle=False)
"""

from __future__ import annotations

import hashlib
import os
import time
from typing import Optional, Sequence

import numpy as np

from . import pack, pack_depth_pro, pack_vggt, weights, weights_depth_pro, weights_vggt
from .common_runtime import *  # noqa: F401,F403  (re-export, as core/common.py does)
from .engine import Engine


def GiB(val):
    return val * 1 << 30


def _parse_synthetic(src: str):
    parts = src.split(":")
    enc = parts[1] if len(parts) > 1 and parts[1] else "vits"
    dtype = parts[2] if len(parts) > 2 and parts[2] else "metric"
    seed = int(parts[3]) if len(parts) > 3 and parts[3] else 1234
    return enc, dtype, seed


def _source_digest(src: str) -> str:
    if src.startswith("synthetic:"):
        return hashlib.sha256(src.encode()).hexdigest()
    h = hashlib.sha256()
    with open(src, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def source_exists(src: str) -> bool:
    return src.startswith("synthetic:") or os.path.exists(src)


def load_checkpoint(path: str) -> dict:
    """Load a state dict without executing anything from the file."""
    if path.endswith(".safetensors"):
        from safetensors.numpy import load_file
        return dict(load_file(path))
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    return {k: v.float().numpy() for k, v in sd.items()}


def is_depth_pro_source(src: str, sd: Optional[dict] = None) -> bool:
    """Depth Pro sources: synthetic:depth_pro[...] or an HF-keyed Depth Pro state dict."""
    if src.startswith("synthetic:"):
        return src.split(":")[1] == "depth_pro"
    return sd is not None and any(k.startswith("depth_pro.encoder.") for k in sd)


def is_vggt_source(src: str, sd: Optional[dict] = None) -> bool:
    """VGGT sources: synthetic:vggt[...] or an upstream-keyed VGGT state dict
    (facebook/VGGT-1B model.pt: aggregator.frame_blocks.*)."""
    if src.startswith("synthetic:"):
        return src.split(":")[1] == "vggt"
    return sd is not None and any(k.startswith("aggregator.frame_blocks.") for k in sd)


def _vggt_config_of(sd: dict) -> dict:
    """The VGGT preset a checkpoint matches (embed dim and block counts)."""
    D = np.asarray(sd["aggregator.camera_token"]).shape[-1]
    nfb = len({k.split(".")[2] for k in sd if k.startswith("aggregator.frame_blocks.")})
    ndb = len({k.split(".")[3] for k in sd if k.startswith("aggregator.patch_embed.blocks.")})
    for preset in weights_vggt.PRESETS:
        cfg = weights_vggt.vggt_config(preset)
        if cfg["embed_dim"] == D and cfg["aa_depth"] == nfb and cfg["depth"] == ndb:
            return cfg
    raise ValueError(f"no VGGT preset matches this checkpoint (dim {D}, {ndb} + {nfb} blocks)")


def _depth_pro_config_of(sd: dict) -> dict:
    """The Depth Pro preset a checkpoint matches (by ViT width / depth and the FOV head)."""
    D = np.asarray(sd["depth_pro.encoder.patch_encoder.model.embeddings.cls_token"]).shape[-1]
    use_fov = any(k.startswith("fov_model.") for k in sd)
    for preset, v in weights_depth_pro.VIT.items():
        cfg = weights_depth_pro.depth_pro_config(preset, use_fov=use_fov)
        if v["embed_dim"] == D and all(k in sd for k in weights_depth_pro.expected_keys(cfg)
                                       if not k.endswith("mask_token")):
            return cfg
    raise ValueError(f"no Depth Pro preset matches this checkpoint (embed dim {D})")


def _infer_encoder(sd: dict) -> str:
    d = np.asarray(sd["pretrained.cls_token"] if "pretrained.cls_token" in sd
                   else sd["module.pretrained.cls_token"]).shape[-1]
    for name, e in weights.ENCODERS.items():
        if e["embed_dim"] == d:
            return name
    raise ValueError(f"no DA-V2 encoder with embed dim {d}")


def _engine_fingerprint(src, precision, workspace_gib, opt_level, obey_precision_constraints,
                        dynamic_input_shapes, encoder, depth_type, max_depth, input_hw,
                        input_format="float32_nchw", frames=None) -> str:
    parts = [_source_digest(src), f"packer={pack.PACKER_VERSION}", f"precision={precision}",
             f"workspace={workspace_gib}", f"opt_level={opt_level}",
             f"obey_precision={obey_precision_constraints}", f"dynamic={dynamic_input_shapes}",
             f"encoder={encoder}", f"depth_type={depth_type}", f"max_depth={max_depth}",
             f"input_hw={tuple(input_hw)}", f"input_format={input_format}", "arch=gfx950"]
    if frames is not None:
        parts.append(f"frames={frames}")
    return "\n".join(parts)


def engine_staleness(engine_file_path, fingerprint_path, fingerprint, source_present):
    """Why the cached engine cannot be reused, or None if it can
    (reference core/common.py:120-138)."""
    if not os.path.exists(engine_file_path):
        return "no engine file"
    if not source_present:
        return None
    if fingerprint is None:
        return None
    if not os.path.exists(fingerprint_path):
        return "no fingerprint recorded"
    with open(fingerprint_path, encoding="utf-8") as f:
        if f.read() != fingerprint:
            return "source or build options changed"
    return None


def get_engine(onnx_file_path, engine_file_path="", precision="fp32", dynamic_input_shapes=None,
               workspace_gib=2, opt_level=None, obey_precision_constraints=False, check_fingerprint=True,
               *, encoder: Optional[str] = None, depth_type: Optional[str] = None,
               max_depth: Optional[float] = None, input_hw: Optional[Sequence[int]] = None,
               input_format: str = "float32_nchw", device: int = 0, frames: Optional[int] = None) -> Engine:
    """Load `engine_file_path` if it matches its source, otherwise pack it.

    `onnx_file_path` keeps the reference's parameter name; it names the
    checkpoint / synthetic spec the engine is packed from.
    `dynamic_input_shapes` = [min, opt, max] input shapes gives a
    dynamic-batch engine whose contexts are sized for max[0] (VGGT: rank-5
    [B, S, 3, H, W] shapes, S fixed).
    `frames` (VGGT): the frame count S the engine is packed for (default 1,
    or the S of the dynamic shapes).
    `precision` (DA-V2): "fp16" -- f16 MFMA operands and activations, the
    residual stream kept in f16 (the reference's fp16 TensorRT engine); "fp32"
    (the reference's default) -- the residual stream, LayerNorm / softmax
    statistics and every accumulation in fp32 with f16 MFMA operands: a
    10-bit mantissa, the precision of the TF32 tensor-core path the
    reference's TensorRT fp32 build takes by default (core/common.py:207-218
    sets no flag that would disable it).  There is no fp32-operand engine.
    Depth Pro / VGGT engines always keep an fp32 residual stream.
    `input_format` "uint8_nhwc" packs the reference's uint8 preamble
    (core/onnx_tools.py:87-219): the input binding becomes "image_u8",
    uint8 [B,H,W,3], normalised on the device.
    """
    if input_format not in pack.INPUT_FORMATS:
        raise ValueError(f"[MDET] input_format must be one of {pack.INPUT_FORMATS}")
    u8 = input_format == "uint8_nhwc"
    src = str(onnx_file_path)
    if precision not in pack.PRECISIONS:
        raise ValueError(f"[MDET] unknown precision {precision!r}")
    if dynamic_input_shapes is not None:
        mn, opt, mx = [tuple(int(v) for v in s) for s in dynamic_input_shapes[:3]]
        if not (mn[1:] == opt[1:] == mx[1:]):
            raise ValueError("[MDET] only the batch dimension may be dynamic")
        if not (1 <= mn[0] <= opt[0] <= mx[0]):
            raise ValueError(f"[MDET] bad batch profile {mn[0]}/{opt[0]}/{mx[0]}")
        if len(mn) == 5:       # VGGT [B, S, 3, H, W]
            input_hw = input_hw or (mn[3], mn[4])
            frames = frames or mn[1]
        else:
            input_hw = input_hw or ((mn[1], mn[2]) if u8 else (mn[2], mn[3]))
        profile = (mn, opt, mx)
    else:
        profile = None
    input_hw = tuple(int(v) for v in (input_hw or (518, 518)))

    sd = None
    if src.startswith("synthetic:"):
        s_enc, s_type, seed = _parse_synthetic(src)
        encoder = encoder or s_enc
        depth_type = depth_type or s_type
    if depth_type is None:
        depth_type = "metric"
    if max_depth is None:
        max_depth = 20.0 if depth_type == "metric" else 1.0

    fingerprint = None
    fingerprint_path = os.path.splitext(engine_file_path)[0] + ".fingerprint" if engine_file_path else ""
    present = source_exists(src)
    if check_fingerprint and present and engine_file_path:
        fingerprint = _engine_fingerprint(src, precision, workspace_gib, opt_level, obey_precision_constraints,
                                          dynamic_input_shapes, encoder, depth_type, max_depth, input_hw,
                                          input_format, frames)

    def build_vggt(sd_, cfg) -> bytes:
        if u8:
            raise ValueError("[MDET] VGGT engines take float32 [B, S, 3, H, W] images (no uint8 preamble)")
        if tuple(input_hw) != (cfg["img"], cfg["img"]):
            raise ValueError(f"[MDET] VGGT packs at its checkpoint grid {cfg['img']}x{cfg['img']}, "
                             f"not {tuple(input_hw)}")
        return pack_vggt.pack_bytes(sd_, cfg, int(frames or 1))

    def build_engine() -> bytes:
        nonlocal sd, encoder
        if not present:
            raise FileNotFoundError(f"[MDET] source {src} not found.")
        if is_depth_pro_source(src):
            parts = src.split(":")
            cfg = weights_depth_pro.depth_pro_config(parts[2] if len(parts) > 2 and parts[2] else "dinov2l16_384")
            sd = weights_depth_pro.synthetic_state_dict(cfg, int(parts[3]) if len(parts) > 3 and parts[3] else 4321)
            return pack_depth_pro.pack_bytes(sd, cfg)
        if is_vggt_source(src):
            parts = src.split(":")
            cfg = weights_vggt.vggt_config(parts[2] if len(parts) > 2 and parts[2] else "vggt_1b")
            sd = weights_vggt.synthetic_state_dict(cfg, int(parts[3]) if len(parts) > 3 and parts[3] else 2468)
            return build_vggt(sd, cfg)
        if not src.startswith("synthetic:"):
            sd = load_checkpoint(src)
            if is_depth_pro_source(src, sd):
                return pack_depth_pro.pack_bytes(sd, _depth_pro_config_of(sd))
            if is_vggt_source(src, sd):
                return build_vggt(sd, _vggt_config_of(sd))
        if src.startswith("synthetic:"):
            cfg = weights.model_config(encoder, depth_type, max_depth)
            sd = weights.synthetic_state_dict(cfg, _parse_synthetic(src)[2])
        else:
            encoder = encoder or _infer_encoder(sd)
            cfg = weights.model_config(encoder, depth_type, max_depth)
        return pack.pack_bytes(sd, cfg, *input_hw, input_format=input_format, precision=precision)

    kw = dict(profile=profile, static_batch=1)
    if engine_file_path:
        stale = engine_staleness(engine_file_path, fingerprint_path, fingerprint, present)
        if stale is None:
            print(f"[MDET] Load engine from file ({engine_file_path})")
            return Engine.from_file(engine_file_path, device, **kw)
        if os.path.exists(engine_file_path):
            print(f"[MDET] Rebuilding engine - {stale}")
    print(f"[MDET] Build engine ({engine_file_path or '<memory>'})")
    t0 = time.time()
    blob = build_engine()
    if engine_file_path:
        pack.write_packed(engine_file_path, blob)
        if fingerprint is not None:
            with open(fingerprint_path, "w", encoding="utf-8") as f:
                f.write(fingerprint)
    print(f"[MDET] Engine build done! ({time.time() - t0:.2f} [sec])")
    if engine_file_path:
        return Engine.from_file(engine_file_path, device, **kw)
    return Engine.from_bytes(blob, device, **kw)

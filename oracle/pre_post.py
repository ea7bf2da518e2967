"""ORACLE -- test infrastructure only.  CPU restatement of the two steps
either side of the DA-V2 engine.

Only `tests/` and `bench.py`'s cpu_baseline leg may import this module, as
the checker; the product path (`monocular_depth_estimation_trt_amd`) never
calls it.

* uint8_preamble: the graph preamble the reference prepends for a uint8
  engine, `core/onnx_tools.py:87-219` (`add_uint8_input`): Cast(u8 -> f32),
  Div(scale), Sub(mean), Div(std) -- all float32, in that order -- then the
  NHWC -> NCHW transpose.  Pinned by the reference's own check,
  `tests/test_uint8_input.py:78-99`, which compares the preamble with the host
  arithmetic `img.astype(float32) / 255; (f - mean) / std` (restated here
  literally; the check is re-run on the same 8x8 seed-0 case in
  tests/test_pre_post_oracle.py).
* postprocess: `models/depth_anything_v2/onnx2trt.py:111-117`:
  F.interpolate(depth[:, None], (src_h, src_w), mode="bilinear",
  align_corners=True), then torch.clamp(min=1e-3, max=1e3).
"""

from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def uint8_preamble(img_u8: np.ndarray, mean=MEAN, std=STD, scale: float = 255.0) -> np.ndarray:
    """uint8 NHWC [B,H,W,3] -> float32 NCHW, the reference preamble's fp32 ops."""
    f = img_u8.astype(np.float32) / np.float32(scale)
    f = (f - np.array(mean, dtype=np.float32)) / np.array(std, dtype=np.float32)
    return np.ascontiguousarray(f.transpose(0, 3, 1, 2))


def postprocess(depth: np.ndarray, src_h: int, src_w: int, lo: float = 1e-3, hi: float = 1e3) -> np.ndarray:
    """fp32 depth [B,h,w] -> [B,src_h,src_w] (bilinear, align_corners=True) clamped to [lo, hi]."""
    d = torch.from_numpy(np.ascontiguousarray(depth, dtype=np.float32))[:, None]
    d = F.interpolate(d, (src_h, src_w), mode="bilinear", align_corners=True)[:, 0]
    return torch.clamp(d, min=lo, max=hi).numpy()


def patch_matrix(x_nchw: np.ndarray) -> np.ndarray:
    """float32 NCHW -> the engine's patch-embed operand [B*ph*pw][672] f16:
    per patch, channel-major 14 rows of 16 (14 pixels + 2 zero columns)."""
    B, C, H, W = x_nchw.shape
    ph, pw = H // 14, W // 14
    p = x_nchw[:, :, :ph * 14, :pw * 14].reshape(B, C, ph, 14, pw, 14).transpose(0, 2, 4, 1, 3, 5)
    out = np.zeros((B, ph, pw, C, 14, 16), np.float16)
    out[..., :14] = p.astype(np.float16)
    return out.reshape(B * ph * pw, C * 14 * 16)

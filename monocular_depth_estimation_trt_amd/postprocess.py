"""On-device depth post-process: the reference's
`models/depth_anything_v2/onnx2trt.py:111-117` -- bilinear
(align_corners=True) resize of the [B,h,w] depth map back to the source
image size, then clamp to [1e-3, 1e3] -- as one HIP kernel
(`mde_op_depth_postprocess`), so the D2H copy carries the final map.
"""

from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from .common_runtime import HostDeviceMem, stream_synchronize


def resize_clamp(d_in: int, batch: int, ih: int, iw: int, d_out: int, oh: int, ow: int,
                 lo: float = 1e-3, hi: float = 1e3, stream: int = 0) -> None:
    """Device pointers in/out (fp32), enqueued on `stream`."""
    _lib.call("mde_op_depth_postprocess", C.c_void_p(int(d_in)), int(batch), int(ih), int(iw),
              C.c_void_p(int(d_out)), int(oh), int(ow), float(lo), float(hi), C.c_void_p(int(stream or 0)))


class DevicePostprocess:
    """Owns the resized map (device + pinned host); `run(d_depth, stream)`
    returns a host view [batch, oh, ow] that the next call overwrites."""

    def __init__(self, batch: int, ih: int, iw: int, oh: int, ow: int, lo: float = 1e-3, hi: float = 1e3):
        self.shape = (int(batch), int(oh), int(ow))
        self.src = (int(ih), int(iw))
        self.lo, self.hi = float(lo), float(hi)
        self.mem: Optional[HostDeviceMem] = HostDeviceMem(batch * oh * ow, np.dtype(np.float32))

    def run(self, d_depth: int, stream: int) -> np.ndarray:
        if self.mem is None:
            raise RuntimeError("DevicePostprocess already freed")
        b, oh, ow = self.shape
        resize_clamp(d_depth, b, self.src[0], self.src[1], self.mem.device, oh, ow, self.lo, self.hi, stream)
        host = self.mem.host
        _lib.call("mde_rt_memcpy_dtoh_async", host.ctypes.data_as(C.c_void_p), C.c_void_p(self.mem.device),
                  host.nbytes, C.c_void_p(int(stream or 0)))
        stream_synchronize(stream)
        return self.mem.host.reshape(self.shape)

    def free(self) -> None:
        if self.mem is not None:
            self.mem.free()
            self.mem = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.free()
        return False


def depth_pro_postprocess(canonical_inverse_depth: np.ndarray, fov_deg: np.ndarray, src_hw, f_px=None):
    """Reference `models/depth_pro/onnx2trt.py:100-117` (outside its timed
    loop): focal length from the predicted FOV (unless given), inverse depth
    rescaled by W / f_px, bilinear (align_corners=False) to the source size
    when it differs from the engine's, depth = 1 / clamp(inv, 1e-4, 1e4).
    Returns (depth [H, W] float32, f_px float)."""
    import torch
    import torch.nn.functional as F
    inv = torch.from_numpy(np.ascontiguousarray(canonical_inverse_depth, dtype=np.float32)).reshape(
        1, 1, *canonical_inverse_depth.shape[-2:])
    H, W = int(src_hw[0]), int(src_hw[1])
    if f_px is None:
        fov = torch.from_numpy(np.asarray(fov_deg, dtype=np.float32).reshape(-1)[:1])
        f_px = 0.5 * W / torch.tan(0.5 * torch.deg2rad(fov.to(torch.float)))
    else:
        f_px = torch.tensor([float(f_px)])
    inv = inv * (W / f_px)
    if (H, W) != tuple(inv.shape[-2:]):
        inv = F.interpolate(inv, size=(H, W), mode="bilinear", align_corners=False)
    depth = 1.0 / torch.clamp(inv, min=1e-4, max=1e4)
    return depth.squeeze().numpy(), float(f_px.squeeze())

"""Helpers for the gpu-marked tests: torch device tensors in, C ABI calls."""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from monocular_depth_estimation_trt_amd import _lib


_KEEP = []  # tensors whose pointers are in flight: freed only after op() syncs


def ptr(t) -> C.c_void_p:
    """Device pointer of t; keeps t alive until the next op() has synchronized
    (a temporary passed inline would otherwise go back to the caching
    allocator and be reused by the next argument's allocation)."""
    if t is None:
        return C.c_void_p(0)
    _KEEP.append(t)
    return C.c_void_p(t.data_ptr())


def stream() -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def op(name: str, *args) -> None:
    try:
        _lib.call(name, *args)
        torch.cuda.synchronize()
    finally:
        _KEEP.clear()


def vt_pos(t):
    """Key permutation of the V^T layout (csrc/mde_device.h vt_pos): bits 2
    and 3 of t swapped."""
    return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1)


def vt_perm(T: int) -> torch.Tensor:
    """Index tensor: storage column of key t, t in [0, T)."""
    return torch.tensor([vt_pos(t) for t in range(T)], dtype=torch.long)


def pad_w(w: torch.Tensor, n_mult: int = 128, k_mult: int = 64) -> torch.Tensor:
    """[N][K] -> f16 [Npad][Kpad] zero-padded device tensor (the packer's layout)."""
    n, k = w.shape
    N = -(-n // n_mult) * n_mult
    K = -(-k // k_mult) * k_mult
    out = torch.zeros(N, K, dtype=torch.float16, device=w.device)
    out[:n, :k] = w.half()
    return out


def conv_w(w: torch.Tensor) -> torch.Tensor:
    """[Cout][Cin][3][3] -> packed [Cout][ky][kx][Cin]."""
    co, ci = w.shape[:2]
    return pad_w(w.permute(0, 2, 3, 1).reshape(co, 9 * ci))


def nhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 3, 1, 2).contiguous()


def close(got: torch.Tensor, ref: torch.Tensor, rtol: float, atol: float, what: str = "") -> None:
    g = got.float().cpu()
    r = ref.float().cpu()
    assert g.shape == r.shape, (what, g.shape, r.shape)
    err = (g - r).abs()
    bound = atol + rtol * r.abs()
    bad = ~(err <= bound)  # NaN counts as bad
    if bad.any():
        i = int(bad.flatten().nonzero()[0])
        raise AssertionError(f"{what}: {int(bad.sum())}/{bad.numel()} elements out of tolerance; "
                             f"max_abs {err.max():.4e}; first bad idx {i}: got {g.flatten()[i]:.6f} "
                             f"ref {r.flatten()[i]:.6f}")


def depth_metrics(got: np.ndarray, ref: np.ndarray) -> dict:
    g = np.asarray(got, np.float64).ravel()
    r = np.asarray(ref, np.float64).ravel()
    d = np.abs(g - r)
    return dict(max_abs=float(d.max()), mean_abs=float(d.mean()),
                rel_mean=float(d.mean() / max(np.abs(r).mean(), 1e-12)),
                corr=float(np.corrcoef(g, r)[0, 1]) if g.size > 1 else 1.0)

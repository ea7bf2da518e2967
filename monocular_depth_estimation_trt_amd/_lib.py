"""ctypes binding of libmde_hip.so (the C ABI declared in include/mde.h).

This is the only door from Python into the HIP engine.  There is no CPU or
PyTorch fallback: if the library is missing or fails to load, every call
raises -- a product path that silently computed on the CPU would void every
parity claim.
"""

from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmde_hip.so")


def use_library(path: str) -> None:
    """Load a tuning-variant build (tools/ablate.py, tools/bench_kernels.py
    --lib) instead of the in-tree product library.  Must run before the first
    lib() call; the product path never calls it (no environment read here:
    the library's dispatch switches, mde.h mde_tuning_*, are the only knobs)."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise RuntimeError(f"libmde_hip already loaded from {LIB_PATH}")
    LIB_PATH = path

c_void_p, c_int, c_float, c_size_t, c_char_p = C.c_void_p, C.c_int, C.c_float, C.c_size_t, C.c_char_p
c_int64 = C.c_int64
P = C.POINTER

MDE_OK = 0
STATUS = {1: "MDE_ERR_ARG", 2: "MDE_ERR_FILE", 3: "MDE_ERR_FORMAT", 4: "MDE_ERR_HIP", 5: "MDE_ERR_NAME",
          6: "MDE_ERR_SHAPE", 7: "MDE_ERR_STATE"}


class mde_io_desc(C.Structure):
    _fields_ = [("name", C.c_char * 64), ("dtype", C.c_int32), ("is_input", C.c_int32),
                ("rank", C.c_int32), ("dims", C.c_int64 * 8)]


class mde_engine_info(C.Structure):
    _fields_ = [("encoder", C.c_char * 16),
                ("embed_dim", C.c_int32), ("depth", C.c_int32), ("num_heads", C.c_int32),
                ("mlp_hidden", C.c_int32), ("patch", C.c_int32),
                ("img_h", C.c_int32), ("img_w", C.c_int32), ("features", C.c_int32),
                ("head_hidden", C.c_int32), ("metric", C.c_int32),
                ("out_channels", C.c_int32 * 4), ("taps", C.c_int32 * 4),
                ("max_depth", C.c_float), ("ln_eps", C.c_float),
                ("max_batch_hint", C.c_int32), ("weight_bytes", C.c_int64),
                ("input_format", C.c_int32), ("family", C.c_int32)]


LAYER_CB = C.CFUNCTYPE(None, c_char_p, c_float, c_void_p)

# name -> argtypes (restype is always int status unless listed in _RESTYPE)
PROTOTYPES = {
    "mde_version": [],
    "mde_last_error": [],
    "mde_tuning_set": [c_char_p, c_int],
    "mde_tuning_get": [c_char_p, P(c_int)],
    "mde_engine_load": [c_char_p, c_int, P(c_void_p)],
    "mde_engine_load_memory": [c_void_p, c_size_t, c_int, P(c_void_p)],
    "mde_engine_destroy": [c_void_p],
    "mde_engine_get_info": [c_void_p, P(mde_engine_info)],
    "mde_engine_num_io": [c_void_p, P(c_int)],
    "mde_engine_io_desc": [c_void_p, c_int, P(mde_io_desc)],
    "mde_engine_profile_shape": [c_void_p, c_char_p, c_int, P(c_int64), P(c_int)],
    "mde_context_create": [c_void_p, c_int, P(c_void_p)],
    "mde_context_destroy": [c_void_p],
    "mde_context_set_tensor_address": [c_void_p, c_char_p, c_void_p],
    "mde_context_set_input_shape": [c_void_p, c_char_p, P(c_int64), c_int],
    "mde_context_get_tensor_shape": [c_void_p, c_char_p, P(c_int64), P(c_int)],
    "mde_context_enqueue": [c_void_p, c_void_p],
    "mde_context_set_graph_mode": [c_void_p, c_int],
    "mde_context_set_profiler": [c_void_p, LAYER_CB, c_void_p],
    "mde_context_workspace_bytes": [c_void_p, P(c_size_t)],
    "mde_rt_device_count": [P(c_int)],
    "mde_rt_set_device": [c_int],
    "mde_rt_device_name": [c_int, c_char_p, c_int],
    "mde_rt_malloc": [P(c_void_p), c_size_t],
    "mde_rt_free": [c_void_p],
    "mde_rt_malloc_host": [P(c_void_p), c_size_t],
    "mde_rt_free_host": [c_void_p],
    "mde_rt_memcpy_htod_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "mde_rt_memcpy_dtoh_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "mde_rt_memcpy_dtod_async": [c_void_p, c_void_p, c_size_t, c_void_p],
    "mde_rt_memset_async": [c_void_p, c_int, c_size_t, c_void_p],
    "mde_rt_stream_create": [P(c_void_p)],
    "mde_rt_stream_destroy": [c_void_p],
    "mde_rt_stream_synchronize": [c_void_p],
    "mde_rt_device_synchronize": [],
    "mde_rt_event_create": [P(c_void_p)],
    "mde_rt_event_destroy": [c_void_p],
    "mde_rt_event_record": [c_void_p, c_void_p],
    "mde_rt_event_elapsed_ms": [P(c_float), c_void_p, c_void_p],
    "mde_op_layernorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_int, c_int, c_void_p],
    "mde_op_layernorm_f16": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_int, c_int, c_void_p],
    "mde_op_linear": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                      c_void_p],
    "mde_op_linear_residual": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                               c_void_p, c_int, c_void_p],
    "mde_op_qkv": [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                   c_void_p, c_void_p],
    "mde_op_linear_residual_f16": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_int, c_void_p, c_void_p],
    "mde_op_linear_lnfold": [c_void_p, c_void_p, c_float, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                             c_int, c_void_p, c_int, c_void_p],
    "mde_op_qkv_lnfold": [c_void_p, c_void_p, c_float, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int,
                          c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "mde_op_attention_ws": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                            c_size_t, c_void_p],
    "mde_op_attention_ws_bytes": [c_int, c_int, c_int],
    "mde_op_attention_cfg": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_char_p,
                             c_void_p, c_size_t, c_void_p],
    "mde_op_attention": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "mde_op_linear32": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                        c_void_p],
    "mde_op_linear_residual32": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_int, c_void_p],
    "mde_op_qkv32": [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                     c_void_p, c_void_p],
    "mde_op_attention32": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "mde_op_conv3x3_32": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                          c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "mde_op_conv_transpose32": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                                c_void_p, c_void_p],
    "mde_op_resize32": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mde_op_patch_embed": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                           c_void_p, c_void_p, c_void_p],
    "mde_op_conv3x3": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                       c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "mde_op_conv3x3_ws": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                          c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, P(c_int), c_void_p],
    "mde_op_linear_ws": [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                         c_void_p, c_size_t, P(c_int), c_void_p],
    "mde_op_conv3x3_up": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                          c_int, c_void_p, c_void_p],
    "mde_op_conv_transpose": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p],
    "mde_op_resize_bilinear": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mde_op_depth_head": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                          c_void_p, c_float, c_int, c_float, c_void_p, c_void_p],
    "mde_op_patch_prep_u8": [c_void_p, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "mde_op_dp_pyramid_patches": [c_void_p, c_int, c_int, c_void_p, c_void_p],
    "mde_op_merge_tokens": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float,
                            c_void_p, c_void_p],
    "mde_op_depth_postprocess": [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_float, c_float,
                                 c_void_p],
    "mde_op_qk_norm_rope": [c_void_p] * 6 + [c_int] * 6 + [c_void_p, c_void_p, c_float, c_float, c_void_p],
    "mde_op_tap_concat_ln": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p,
                             c_void_p],
}
_RESTYPE = {"mde_last_error": c_char_p, "mde_op_attention_ws_bytes": c_size_t}

_lib = None
_lock = threading.Lock()


class MDEError(RuntimeError):
    """A non-zero status from libmde_hip (mirrors core/common_runtime.py:41-56)."""

    def __init__(self, fn: str, code: int, msg: str):
        self.code = code
        super().__init__(f"{fn} failed ({STATUS.get(code, code)}): {msg}")


def hip_runtimes() -> list:
    """The distinct libamdhip64 images mapped into this process (from
    /proc/self/maps; empty where that is not readable)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) == 6 and "libamdhip64" in os.path.basename(parts[5].strip()):
                    paths.add(os.path.realpath(parts[5].strip()))
    except OSError:
        return []
    return sorted(paths)


def check_single_runtime() -> None:
    """Raise if two HIP runtimes are mapped into this process.

    Root cause (established on this image): PyTorch-ROCm's bundled
    torch/lib/libamdhip64.so and ROCm's /opt/rocm/lib/libamdhip64.so.7 both
    carry the SONAME libamdhip64.so.7.  libmde_hip.so NEEDs that soname, so
    when torch is loaded first the dynamic loader binds libmde_hip to torch's
    runtime (one runtime: torch's streams and ours are the same objects).
    When libmde_hip is loaded first it maps ROCm's copy, and a later torch
    import NEEDs "libamdhip64.so" -- no soname match -- and maps a second
    runtime: each initialises its own HSA runtime, ours then sees no device
    (hipSetDevice: no ROCm-capable device), and a hipStream_t that torch hands
    across the ABI would belong to the other runtime.  Nothing works reliably
    in that state, so fail loudly instead."""
    rts = hip_runtimes()
    if len(rts) > 1:
        raise ImportError(
            "two HIP runtimes are loaded in this process (" + ", ".join(rts) + "): libmde_hip.so was loaded "
            "before PyTorch's bundled HIP runtime.  Import torch (and call torch.cuda.is_available()) before "
            "loading libmde_hip.so, or do not load torch in a process that uses libmde_hip.so directly.")


def lib() -> C.CDLL:
    """Load libmde_hip.so once; raise loudly if it is not there."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"libmde_hip.so not found at {LIB_PATH}. Build it first: "
                    f"python -c 'import __graft_entry__ as g; g.build()' (or "
                    f"python -m monocular_depth_estimation_trt_amd._build). There is no CPU fallback.")
            # One HIP runtime per process (check_single_runtime): when torch
            # is importable, bring its bundled runtime up first so that
            # libmde_hip binds to it and the streams torch hands over are the
            # runtime's own.
            try:
                import torch
                torch.cuda.is_available()
            except ImportError:
                pass
            L = C.CDLL(LIB_PATH)
            check_single_runtime()
            for name, args in PROTOTYPES.items():
                f = getattr(L, name)
                f.argtypes = args
                f.restype = _RESTYPE.get(name, c_int)
            _lib = L
    return _lib


def last_error() -> str:
    m = lib().mde_last_error()
    return m.decode(errors="replace") if m else ""


def call(name: str, *args) -> None:
    """Invoke an ABI function, raising MDEError on a non-zero status."""
    rc = getattr(lib(), name)(*args)
    if rc != MDE_OK:
        raise MDEError(name, rc, last_error())


TUNING = ("splitk", "lnfold", "conv_narrow", "upconv", "gemm256", "deep64", "w8small", "conv_persist", "panel",
          "panel32", "narrow_resid", "attn16", "splitk_fused", "attn_tail", "resize_fold")
TUNING_DEFAULT = {"panel32": 0, "splitk_fused": 0, "attn_tail": 2}  # the library's defaults where not 1 (tuning.hip kKnobs)


def get_tuning(name: str) -> int:
    v = c_int()
    call("mde_tuning_get", name.encode(), C.byref(v))
    return v.value


def set_tuning(name: str, value: int) -> None:
    """Set a dispatch switch of the library (include/mde.h mde_tuning_set)."""
    rc = lib().mde_tuning_set(name.encode(), int(value))
    if rc != MDE_OK:
        raise ValueError(f"mde_tuning_set({name!r}, {value}) failed ({STATUS.get(rc, rc)}): "
                         f"known switches {TUNING}")


@contextlib.contextmanager
def tuning(**switches):
    """Temporarily set dispatch switches: `with tuning(splitk=0): ...`."""
    old = {k: get_tuning(k) for k in switches}
    try:
        for k, v in switches.items():
            set_tuning(k, v)
        yield
    finally:
        for k, v in old.items():
            set_tuning(k, v)


def exported_symbols():
    return list(PROTOTYPES)

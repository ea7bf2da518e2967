"""Engine / ExecutionContext: the TensorRT-shaped Python face of libmde_hip.

The reference drives `trt.ICudaEngine` and `trt.IExecutionContext`
(`models/depth_anything_v2/onnx2trt.py:93-107`, `core/common_runtime.py:
131-175, 268-275`).  These classes expose the same members those call sites
use -- num_io_tensors, get_tensor_name/shape/dtype/mode,
get_tensor_profile_shape, create_execution_context, set_tensor_address,
set_input_shape, execute_async_v3, the `profiler` attribute and the context
manager protocol -- over the C ABI (include/mde.h).
"""

from __future__ import annotations

import ctypes as C
import enum
import weakref
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import call


class DataType(enum.IntEnum):
    """Subset of tensorrt.DataType (same values)."""
    FLOAT = 0
    HALF = 1
    UINT8 = 5

    @property
    def itemsize(self) -> int:
        return {DataType.FLOAT: 4, DataType.HALF: 2, DataType.UINT8: 1}[self]


class TensorIOMode(enum.IntEnum):
    NONE = 0
    INPUT = 1
    OUTPUT = 2


def nptype(dt: DataType):
    """tensorrt.nptype analogue."""
    return {DataType.FLOAT: np.float32, DataType.HALF: np.float16, DataType.UINT8: np.uint8}[DataType(dt)]


def volume(shape: Sequence[int]) -> int:
    """tensorrt.volume analogue (product of dims; a -1 dim gives a negative)."""
    v = 1
    for s in shape:
        v *= int(s)
    return v


class IProfiler:
    """Base class mirroring trt.IProfiler: override report_layer_time."""

    def report_layer_time(self, layer_name: str, ms: float) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class Engine:
    """A loaded packed engine on one device (trt.ICudaEngine analogue).

    `profile` = (min, opt, max) input shapes of the dynamic-batch profile, or
    None for a static engine whose batch is fixed at `static_batch`.
    """

    def __init__(self, handle: int, device: int, profile: Optional[Tuple[Sequence[int], ...]] = None,
                 static_batch: int = 1, path: str = ""):
        self._h = C.c_void_p(handle)
        self.device = device
        self.path = path
        self._contexts = weakref.WeakSet()
        # torch imported after libmde_hip was loaded maps a second HIP runtime
        # (_lib.check_single_runtime): refuse to run in that state -- and free
        # the packed weights the handle already holds on the device
        try:
            _lib.check_single_runtime()
        except Exception:
            self.destroy()
            raise
        self._profile = tuple(tuple(int(v) for v in s) for s in profile) if profile else None
        self._static_batch = int(static_batch)
        info = _lib.mde_engine_info()
        call("mde_engine_get_info", self._h, C.byref(info))
        self.info = info
        n = C.c_int()
        call("mde_engine_num_io", self._h, C.byref(n))
        self._io = []
        for i in range(n.value):
            d = _lib.mde_io_desc()
            call("mde_engine_io_desc", self._h, i, C.byref(d))
            self._io.append((d.name.decode(), DataType(d.dtype), bool(d.is_input),
                             tuple(int(d.dims[k]) for k in range(d.rank))))

    # ---- loading ----
    @classmethod
    def from_file(cls, path: str, device: int = 0, **kw) -> "Engine":
        h = C.c_void_p()
        call("mde_engine_load", path.encode(), int(device), C.byref(h))
        return cls(h.value, device, path=path, **kw)

    @classmethod
    def from_bytes(cls, blob: bytes, device: int = 0, **kw) -> "Engine":
        h = C.c_void_p()
        # the bytes object itself is the argument (ctypes passes its buffer):
        # a create_string_buffer copy passed through C.cast forms a reference
        # cycle, and the whole packed blob (53 MB ViT-S, 671 MB ViT-L) then
        # waited for a cyclic-GC pass to be freed -- which landed inside the
        # batch-1 timed loop as a 7.7 ms (ViT-S) / ~76 ms (ViT-L) sample
        # (bench.py b1_gc_in_loop, gpurun_out/r4s1)
        blob = bytes(blob) if not isinstance(blob, bytes) else blob
        call("mde_engine_load_memory", blob, len(blob), int(device), C.byref(h))
        return cls(h.value, device, **kw)

    @property
    def handle(self) -> C.c_void_p:
        if not self._h:
            raise RuntimeError("engine already destroyed")
        return self._h

    # ---- introspection (ICudaEngine) ----
    @property
    def num_io_tensors(self) -> int:
        return len(self._io)

    def get_tensor_name(self, i: int) -> str:
        return self._io[i][0]

    def _find(self, name: str):
        for rec in self._io:
            if rec[0] == name:
                return rec
        raise KeyError(f"no tensor named {name!r}; have {[r[0] for r in self._io]}")

    def get_tensor_dtype(self, name: str) -> DataType:
        return self._find(name)[1]

    def get_tensor_mode(self, name: str) -> TensorIOMode:
        return TensorIOMode.INPUT if self._find(name)[2] else TensorIOMode.OUTPUT

    def get_tensor_shape(self, name: str) -> Tuple[int, ...]:
        dims = list(self._find(name)[3])
        dims[0] = -1 if self._profile else self._static_batch
        return tuple(dims)

    def get_tensor_profile_shape(self, name: str, profile_index: int) -> List[Tuple[int, ...]]:
        if profile_index != 0:
            raise IndexError(f"engine has one optimization profile; got index {profile_index}")
        dims = list(self._find(name)[3])
        if self._profile:
            bs = [s[0] for s in self._profile]
        else:
            bs = [self._static_batch] * 3
        return [tuple([b] + dims[1:]) for b in bs]

    @property
    def max_batch(self) -> int:
        return self._profile[2][0] if self._profile else self._static_batch

    @property
    def input_hw(self) -> Tuple[int, int]:
        return int(self.info.img_h), int(self.info.img_w)

    @property
    def input_name(self) -> str:
        """"input" (float32 NCHW) or "image_u8" (uint8 NHWC engines)."""
        return next(r[0] for r in self._io if r[2])

    @property
    def input_format(self) -> str:
        return "uint8_nhwc" if int(self.info.input_format) == 1 else "float32_nchw"

    def create_execution_context(self) -> "ExecutionContext":
        return ExecutionContext(self)

    # ---- lifetime ----
    def destroy(self) -> None:
        if self._h:
            for ctx in list(self._contexts):   # a context must not outlive its engine
                ctx.destroy()
            _lib.lib().mde_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()
        return False

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class ExecutionContext:
    """trt.IExecutionContext analogue; owns the activation workspace."""

    def __init__(self, engine: Engine, max_batch: Optional[int] = None):
        self.engine = engine
        h = C.c_void_p()
        call("mde_context_create", engine.handle, int(max_batch or engine.max_batch), C.byref(h))
        self._h = h
        engine._contexts.add(self)
        self._profiler = None
        self._cb = None
        if not engine._profile:
            name = engine.input_name
            self.set_input_shape(name, (engine._static_batch,) + tuple(engine._find(name)[3][1:]))

    @property
    def handle(self) -> C.c_void_p:
        if not self._h:
            raise RuntimeError("context already destroyed")
        return self._h

    def set_tensor_address(self, name: str, ptr: int) -> bool:
        call("mde_context_set_tensor_address", self.handle, name.encode(), C.c_void_p(int(ptr)))
        return True

    def set_input_shape(self, name: str, shape: Sequence[int]) -> bool:
        arr = (C.c_int64 * len(shape))(*[int(s) for s in shape])
        call("mde_context_set_input_shape", self.handle, name.encode(), arr, len(shape))
        return True

    def get_tensor_shape(self, name: str) -> Tuple[int, ...]:
        dims = (C.c_int64 * 8)()
        rank = C.c_int()
        call("mde_context_get_tensor_shape", self.handle, name.encode(), dims, C.byref(rank))
        return tuple(int(dims[i]) for i in range(rank.value))

    def execute_async_v3(self, stream_handle) -> bool:
        call("mde_context_enqueue", self.handle, C.c_void_p(int(stream_handle) if stream_handle else 0))
        return True

    def set_graph_mode(self, enable: bool) -> None:
        call("mde_context_set_graph_mode", self.handle, 1 if enable else 0)

    @property
    def workspace_bytes(self) -> int:
        n = C.c_size_t()
        call("mde_context_workspace_bytes", self.handle, C.byref(n))
        return n.value

    # IExecutionContext.profiler: any object with report_layer_time(name, ms)
    @property
    def profiler(self):
        return self._profiler

    @profiler.setter
    def profiler(self, prof) -> None:
        self._profiler = prof
        if prof is None:
            self._cb = None
            call("mde_context_set_profiler", self.handle, _lib.LAYER_CB(), None)
            return

        def _cb(name, ms, _user):
            prof.report_layer_time(name.decode(), float(ms))

        self._cb = _lib.LAYER_CB(_cb)
        call("mde_context_set_profiler", self.handle, self._cb, None)

    def destroy(self) -> None:
        if self._h:
            _lib.lib().mde_context_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()
        return False

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

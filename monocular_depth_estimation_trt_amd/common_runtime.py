"""Buffers, copies, stage timing and do_inference -- the drop-in for the
reference's `core/common_runtime.py` (:59-275), on HIP instead of cudart.

Same names, same argument meaning, same error behaviour:
  HostDeviceMem(size, dtype)  pinned host + device pair (:59-108)
  allocate_buffers(engine, output_shape=None, profile_idx=None)
        -> (inputs, outputs, bindings, stream)        (:131-175)
  free_buffers(inputs, outputs, stream)               (:179-182)
  memcpy_host_to_device / memcpy_device_to_host       (:186-193)
  StageTimer                                          (:196-238)
  _do_inference_base / do_inference                   (:241-275)
A failing runtime call raises RuntimeError with the HIP error text
(`cuda_call`/`check_cuda_err`, :41-56); size mismatches raise ValueError.
The memory helpers go through libmde_hip's mde_rt_* ABI, so this module needs
neither torch nor a vendor Python binding.
"""

from __future__ import annotations

import ctypes as C
from typing import List, Optional, Union

import numpy as np

from . import _lib
from .engine import DataType, Engine, TensorIOMode, nptype, volume

__all__ = ["HostDeviceMem", "allocate_buffers", "free_buffers", "memcpy_host_to_device",
           "memcpy_device_to_host", "StageTimer", "do_inference", "_do_inference_base", "hip_call",
           "stream_create", "stream_destroy", "stream_synchronize", "volume", "nptype", "DataType",
           "TensorIOMode"]


def hip_call(name: str, *args) -> None:
    """cuda_call analogue: run one mde_rt_* function, RuntimeError on failure."""
    _lib.call(name, *args)


def stream_create() -> int:
    s = C.c_void_p()
    hip_call("mde_rt_stream_create", C.byref(s))
    return int(s.value or 0)


def stream_destroy(stream: int) -> None:
    hip_call("mde_rt_stream_destroy", C.c_void_p(stream))


def stream_synchronize(stream: int) -> None:
    hip_call("mde_rt_stream_synchronize", C.c_void_p(stream))


class HostDeviceMem:
    """Pair of pinned host memory (wrapped as numpy) and device memory."""

    def __init__(self, size: int, dtype: Optional[np.dtype] = None):
        dtype = np.dtype(dtype or np.uint8)
        nbytes = int(size) * dtype.itemsize
        hptr = C.c_void_p()
        hip_call("mde_rt_malloc_host", C.byref(hptr), max(nbytes, 1))
        byte_ptr = C.cast(hptr, C.POINTER(C.c_uint8))
        self._host = np.ctypeslib.as_array(byte_ptr, (nbytes,)).view(dtype)
        dptr = C.c_void_p()
        try:
            hip_call("mde_rt_malloc", C.byref(dptr), max(nbytes, 1))
        except Exception:
            hip_call("mde_rt_free_host", hptr)
            raise
        self._hptr = int(hptr.value)
        self._device = int(dptr.value)
        self._nbytes = nbytes

    @property
    def host(self) -> np.ndarray:
        return self._host

    @host.setter
    def host(self, data: Union[np.ndarray, bytes]):
        if isinstance(data, np.ndarray):
            if data.size > self.host.size:
                raise ValueError(
                    f"Tried to fit an array of size {data.size} into host memory of size {self.host.size}")
            np.copyto(self.host[:data.size], data.flat, casting="safe")
        else:
            assert self.host.dtype == np.uint8
            self.host[:self.nbytes] = np.frombuffer(data, dtype=np.uint8)

    @property
    def device(self) -> int:
        return self._device

    @property
    def nbytes(self) -> int:
        return self._nbytes

    def __str__(self):
        return f"Host:\n{self.host}\nDevice:\n{self.device}\nSize:\n{self.nbytes}\n"

    __repr__ = __str__

    def free(self):
        if self._device:
            hip_call("mde_rt_free", C.c_void_p(self._device))
            self._device = 0
        if self._hptr:
            hip_call("mde_rt_free_host", C.c_void_p(self._hptr))
            self._hptr = 0


def _resolve_shape_override(binding, shape, size, output_shape):
    """Shape to allocate for `binding`, or None to keep the engine's.
    `output_shape`: dict {name: shape} (looked up by name) or one shape, used
    only when the engine's own shape is unusable (dynamic or volume <= 1)."""
    if output_shape is None:
        return None
    if isinstance(output_shape, dict):
        return output_shape.get(binding)
    engine_shape_usable = all(s >= 0 for s in shape) and size > 1
    return None if engine_shape_usable else output_shape


def allocate_buffers(engine: Engine, output_shape=None, profile_idx: Optional[int] = None):
    """Allocate pinned-host/device buffers for every IO tensor of `engine`.
    With a dynamic-batch engine pass profile_idx to size for the profile max."""
    inputs, outputs, bindings = [], [], []
    stream = stream_create()
    for i in range(engine.num_io_tensors):
        binding = engine.get_tensor_name(i)
        shape = (engine.get_tensor_shape(binding) if profile_idx is None
                 else engine.get_tensor_profile_shape(binding, profile_idx)[-1])
        if not all(s >= 0 for s in shape) and profile_idx is None:
            raise ValueError(f"Binding {binding} has dynamic shape, but no profile was specified.")
        size = volume(shape)
        override = _resolve_shape_override(binding, shape, size, output_shape)
        if override is not None:
            size = volume(override)
        mem = HostDeviceMem(size, np.dtype(nptype(engine.get_tensor_dtype(binding))))
        bindings.append(int(mem.device))
        if engine.get_tensor_mode(binding) == TensorIOMode.INPUT:
            inputs.append(mem)
        else:
            outputs.append(mem)
    return inputs, outputs, bindings, stream


def free_buffers(inputs: List[HostDeviceMem], outputs: List[HostDeviceMem], stream: int):
    for mem in inputs + outputs:
        mem.free()
    stream_destroy(stream)


def memcpy_host_to_device(device_ptr: int, host_arr: np.ndarray):
    nbytes = host_arr.size * host_arr.itemsize
    hip_call("mde_rt_memcpy_htod_async", C.c_void_p(device_ptr), host_arr.ctypes.data_as(C.c_void_p), nbytes,
             None)
    hip_call("mde_rt_device_synchronize")


def memcpy_device_to_host(host_arr: np.ndarray, device_ptr: int):
    nbytes = host_arr.size * host_arr.itemsize
    hip_call("mde_rt_memcpy_dtoh_async", host_arr.ctypes.data_as(C.c_void_p), C.c_void_p(device_ptr), nbytes,
             None)
    hip_call("mde_rt_device_synchronize")


class StageTimer:
    """hipEvents between the three phases of one inference (h2d / compute /
    d2h), recorded on the inference stream; GPU-side durations that do not
    sum to the wall clock (launch overhead and the final sync are outside)."""

    STAGES = ("h2d_ms", "compute_ms", "d2h_ms")

    def __init__(self):
        self._events = []
        for _ in range(4):
            e = C.c_void_p()
            hip_call("mde_rt_event_create", C.byref(e))
            self._events.append(e)
        self.last = {}

    def mark(self, i, stream):
        hip_call("mde_rt_event_record", self._events[i], C.c_void_p(stream))

    def read(self):
        """Milliseconds per phase. Only valid after the stream has synchronized."""
        out = {}
        for i, name in enumerate(self.STAGES):
            ms = C.c_float()
            hip_call("mde_rt_event_elapsed_ms", C.byref(ms), self._events[i], self._events[i + 1])
            out[name] = float(ms.value)
        self.last = out
        return out

    def free(self):
        for e in self._events:
            hip_call("mde_rt_event_destroy", e)
        self._events = []


def _do_inference_base(inputs, outputs, stream, execute_async_func, timer=None):
    s = C.c_void_p(stream)
    if timer is not None:
        timer.mark(0, stream)
    for inp in inputs:
        hip_call("mde_rt_memcpy_htod_async", C.c_void_p(inp.device), inp.host.ctypes.data_as(C.c_void_p),
                 inp.nbytes, s)
    if timer is not None:
        timer.mark(1, stream)
    execute_async_func()
    if timer is not None:
        timer.mark(2, stream)
    for out in outputs:
        hip_call("mde_rt_memcpy_dtoh_async", out.host.ctypes.data_as(C.c_void_p), C.c_void_p(out.device),
                 out.nbytes, s)
    if timer is not None:
        timer.mark(3, stream)
    hip_call("mde_rt_stream_synchronize", s)
    if timer is not None:
        timer.read()
    return [out.host for out in outputs]


def do_inference(context, engine, bindings, inputs, outputs, stream, timer=None):
    """H2D copy, enqueue the engine, D2H copy, sync; returns host views that the
    next call overwrites (copy them to keep them)."""
    def execute_async_func():
        context.execute_async_v3(stream_handle=stream)
    for i in range(engine.num_io_tensors):
        context.set_tensor_address(engine.get_tensor_name(i), bindings[i])
    return _do_inference_base(inputs, outputs, stream, execute_async_func, timer)

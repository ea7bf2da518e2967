"""The C-ABI library loads and exports every symbol include/mde.h declares
(no compute calls: runs without a GPU)."""

import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mde.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mde_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib_path():
    from monocular_depth_estimation_trt_amd import _build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        _build.build_library()
    return _lib.LIB_PATH


def test_header_declares_the_api():
    fns = declared_functions()
    for must in ("mde_engine_load", "mde_context_create", "mde_context_enqueue", "mde_context_set_tensor_address",
                 "mde_rt_malloc_host", "mde_op_attention", "mde_last_error", "mde_version"):
        assert must in fns


def test_every_declared_symbol_is_exported(lib_path):
    lib = ctypes.CDLL(lib_path)
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_binding_covers_the_header(lib_path):
    from monocular_depth_estimation_trt_amd import _lib
    assert set(declared_functions()) == set(_lib.PROTOTYPES), \
        set(declared_functions()) ^ set(_lib.PROTOTYPES)
    L = _lib.lib()
    ver = int(re.search(r"#define MDE_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert L.mde_version() == ver


def test_info_struct_matches_header():
    """ctypes mirror of mde_engine_info / mde_io_desc has every header field, in order."""
    from monocular_depth_estimation_trt_amd import _lib
    txt = open(HEADER).read()
    body = re.search(r"typedef struct \{([^}]*)\} mde_engine_info;", txt).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"([a-z_0-9]+)(?:\[\d+\])?\s*[,;]", body)
    assert names == [f[0] for f in _lib.mde_engine_info._fields_]


def test_errors_without_gpu_are_reported_not_crashed(lib_path):
    """Host-side argument checks answer before any device call."""
    from monocular_depth_estimation_trt_amd import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.mde_engine_load(b"/nonexistent/engine.mdeng", 0, ctypes.byref(h))
    assert rc == 2 and b"cannot open" in L.mde_last_error()
    rc = L.mde_engine_load_memory(b"NOTAPACK" + b"\0" * 400, 408, 0, ctypes.byref(h))
    assert rc == 3 and b"magic" in L.mde_last_error()
    rc = L.mde_op_linear(None, 8, None, 64, 4, 4, 8, None, 0, None, 4, None)
    assert rc == 1

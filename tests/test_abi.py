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
    from monocular_depth_estimation_trt_amd import _lib
    lib = _lib.lib()  # (a bare ctypes.CDLL before torch would map a second HIP runtime)
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


def test_tuning_switches(lib_path):
    """The library's dispatch switches (include/mde.h mde_tuning_set/_get):
    defaults, range and name checks, and the context manager restores."""
    from monocular_depth_estimation_trt_amd import _lib
    L = _lib.lib()
    for name in _lib.TUNING:
        assert _lib.get_tuning(name) == _lib.TUNING_DEFAULT.get(name, 1), name
    v = ctypes.c_int()
    assert L.mde_tuning_get(b"no_such_switch", ctypes.byref(v)) == 5
    assert L.mde_tuning_set(b"splitk", 2) == 1
    assert L.mde_tuning_set(b"gemm256", 2) == 0 and _lib.get_tuning("gemm256") == 2
    _lib.set_tuning("gemm256", 1)
    with _lib.tuning(splitk=0, deep64=0):
        assert _lib.get_tuning("splitk") == 0 and _lib.get_tuning("deep64") == 0
    assert _lib.get_tuning("splitk") == 1 and _lib.get_tuning("deep64") == 1
    with pytest.raises(ValueError):
        _lib.set_tuning("lnfold", 7)


def _run_py(code, env=None):
    import subprocess
    import sys
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600, env=e)
    return r.returncode, r.stdout + r.stderr


def test_tuning_reads_environment_once(lib_path):
    rc, out = _run_py("from monocular_depth_estimation_trt_amd import _lib\n"
                      "print(_lib.get_tuning('splitk'), _lib.get_tuning('gemm256'), _lib.get_tuning('w8small'))",
                      {"MDE_SPLITK": "0", "MDE_GEMM256": "2", "MDE_W8SMALL": "bogus"})
    assert rc == 0, out
    vals = [l for l in out.splitlines() if not l.startswith("[mde]")][-1]
    assert vals.split() == ["0", "2", "1"], out
    assert "MDE_W8SMALL=bogus ignored" in out, out


def test_one_hip_runtime_when_torch_comes_first(lib_path):
    """_lib.lib() brings torch's bundled HIP runtime up first; libmde_hip then
    binds to it (same SONAME), so exactly one runtime is mapped and it is
    torch's -- the runtime that owns the streams torch passes in."""
    rc, out = _run_py("from monocular_depth_estimation_trt_amd import _lib\n"
                      "_lib.lib()\n"
                      "print('RT', _lib.hip_runtimes())")
    assert rc == 0, out
    line = [l for l in out.splitlines() if l.startswith("RT ")][-1]
    rts = eval(line[3:])
    assert len(rts) == 1 and "torch" in rts[0], out


def test_two_hip_runtimes_are_refused(lib_path):
    """libmde_hip loaded before torch maps ROCm's runtime; a later torch
    import maps its own second copy (the r3 smoke failure).  The binding
    refuses that state with an explanation instead of failing in hipSetDevice."""
    rc, out = _run_py("import ctypes\n"
                      f"ctypes.CDLL({lib_path!r})\n"
                      "import torch\n"
                      "torch.cuda.is_available()\n"
                      "from monocular_depth_estimation_trt_amd import _lib\n"
                      "try:\n"
                      "    _lib.lib()\n"
                      "except ImportError as e:\n"
                      "    print('REFUSED', e)\n")
    assert rc == 0, out
    assert "REFUSED two HIP runtimes" in out, out


@pytest.mark.parametrize("tpad, heads, msg", [(40, 6, b"% 16"), (36, 6, b"tokens_pad < tokens"), (48, 0, b"> 0")])
def test_qkv_ops_reject_bad_geometry(lib_path, tpad, heads, msg):
    """V^T stores key t at vt_pos(t) (bits 2 and 3 swapped), so a
    tokens_pad that is not a multiple of 16 would spill the last key group into
    the next row.  Both qkv entry points refuse it before touching the device."""
    from monocular_depth_estimation_trt_amd import _lib
    lib = _lib.lib()
    p = 4096  # never dereferenced: the geometry check runs first
    rc = lib.mde_op_qkv(p, p, 384, p, 1, 37, heads, tpad, 0.125, p, p, p, None)
    assert rc != 0 and msg in lib.mde_last_error()
    rc = lib.mde_op_qkv_lnfold(p, p, 1e-6, p, 384, p, p, 1, 37, heads, tpad, 0.125, p, p, p, None)
    assert rc != 0 and msg in lib.mde_last_error()

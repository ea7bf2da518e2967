"""Build libmde_hip.so in-tree with hipcc for gfx950 (no JIT cache, no setup.py).

The .so lands next to this file so it travels with the repository snapshot to
the GPU box and is the file the Python layer loads (`_lib.py`).
"""

from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(HERE, "libmde_hip.so")
OBJDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("MDE_OFFLOAD_ARCH", "gfx950")
SOURCES = ["gemm.hip", "conv.hip", "attention.hip", "elementwise.hip", "engine.hip",
           "depth_pro.hip", "depth_pro_ops.hip", "gemm256.hip", "gemm_panel.hip", "vggt.hip", "vggt_ops.hip", "tuning.hip", "fp32.hip"]
# attention / conv: no NaN inputs by construction (masked keys are -inf, never
# NaN; activations finite); lets fmaxf / the ReLUs lower to a bare v_max
# without canonicalising moves (v_pk_max_f16 x, x before every f16 ReLU)
PER_FILE = {"attention.hip": ["-fno-honor-nans"], "conv.hip": ["-fno-honor-nans"]}
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wno-unused-result", "-I", CSRC, "-I", INCLUDE]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmde_hip.so)")


def _digest() -> str:
    h = hashlib.sha256()
    for name in sorted(os.listdir(CSRC)):
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode())
            h.update(f.read())
    with open(os.path.join(INCLUDE, "mde.h"), "rb") as f:
        h.update(f.read())
    # flags without the checkout's absolute paths: the same tree at another
    # path (the GPU box's copy) is the same build
    h.update(" ".join(FLAGS).replace(ROOT, "<root>").encode())
    h.update(repr(sorted(PER_FILE.items())).encode())
    return h.hexdigest()


def _stamp_path() -> str:
    return LIB + ".srcsha"


def up_to_date() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(_stamp_path()):
        return False
    with open(_stamp_path()) as f:
        return f.read().strip() == _digest()


def build_library(force: bool = False, verbose: bool = True, out: str = "", defines=()) -> str:
    """Build the library; `out`/`defines` build a tuning variant elsewhere
    (e.g. defines=("MDE_GEMM_BK=32",)) without touching the product .so: a
    variant with defines but no `out` goes to build/var/lib_<hash>.so."""
    variant = bool(out or defines)
    if defines and not out:
        out = os.path.join(ROOT, "build", "var", "lib_" + hashlib.sha1("|".join(defines).encode()).hexdigest()[:10] + ".so")
        os.makedirs(os.path.dirname(out), exist_ok=True)
    if variant and os.path.abspath(out) == os.path.abspath(LIB):
        raise ValueError("a tuning variant must not overwrite the product libmde_hip.so")
    if not variant and not force and up_to_date():
        return LIB
    cc = hipcc()
    objdir = OBJDIR if not variant else os.path.join(OBJDIR, "variant_" + hashlib.sha1(
        (out + "|".join(defines)).encode()).hexdigest()[:10])
    os.makedirs(objdir, exist_ok=True)
    dflags = [f"-D{d}" for d in defines]
    target = out or LIB
    os.makedirs(os.path.dirname(os.path.abspath(target)), exist_ok=True)

    def compile_one(src: str) -> str:
        obj = os.path.join(objdir, src + ".o")
        cmd = [cc, *FLAGS, *PER_FILE.get(src, []), *dflags, "-c", os.path.join(CSRC, src), "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-6000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = target + ".tmp"
    cmd = [cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, target)
    if not variant:
        with open(_stamp_path(), "w") as f:
            f.write(_digest())
    if verbose:
        print(f"[mde] built {target}", file=sys.stderr)
    return target


if __name__ == "__main__":
    build_library(force="--force" in sys.argv)

"""Every LDS-DMA in the product library uses the 64-bit-address form
(`global_load_lds_dwordx4 v[a:b], off`).  The SADDR (`v, s[..]`) and MUBUF
(`buffer_load ... lds`) forms take a 32-bit offset register; with them a
ds_read destination reusing that register gave nondeterministic outputs in
round 4's fused-MLP experiment (tools/dma_hazard_scan.py).
CPU only: disassembles the device code of the in-tree build's objects."""
import glob
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from monocular_depth_estimation_trt_amd import _build

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="ROCm llvm-objdump absent")
def test_product_lds_dma_uses_the_64bit_address_form():
    _build.build_library(verbose=False)
    seen = 0
    for src in _build.SOURCES:
        obj = os.path.join(_build.OBJDIR, src + ".o")
        d = tempfile.mkdtemp()
        try:
            c = os.path.join(d, os.path.basename(obj))
            shutil.copy(obj, c)
            subprocess.run([OBJDUMP, "--offloading", c], capture_output=True, check=True)
            dev = [f for f in glob.glob(c + ".*") if f.endswith("gfx950")]
            if not dev:
                continue
            txt = subprocess.run([OBJDUMP, "-d", dev[0]], capture_output=True, text=True, check=True).stdout
        finally:
            shutil.rmtree(d)
        seen += len(re.findall(r"global_load_lds_dword\w*", txt))
        assert not re.findall(r"global_load_lds_dword\w*\s+v\d+, s\[", txt), src
        assert not re.findall(r"buffer_load_\w+[^\n]*\blds\b", txt), src
    assert seen > 0

"""Every LDS-DMA in the product library uses the 64-bit-address form
(`global_load_lds_dwordx4 v[a:b], off`), except the panel GEMM
(gemm_panel.hip), whose DMAs take the SADDR form (`v, s[..]`: SGPR base + a
32-bit VGPR offset, so no 64-bit address pair is live across its loop).  A
ds_read destination reusing the offset register of an in-flight DMA was the
suspect of round 4's nondeterministic fused-MLP experiment; the round-5 probe
(tools/dma_war_probe.hip, profiles/r05_dma_war_probe.json) found the SADDR
form as safe as the vaddr form, and the second test below requires that no
reuse site of a non-vaddr form exists anyway.  The MUBUF `... lds` form stays
out.  CPU only: disassembles the device code of the in-tree build's objects."""
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
        if src != "gemm_panel.hip":
            assert not re.findall(r"global_load_lds_dword\w*\s+v\d+, s\[", txt), src
        assert not re.findall(r"buffer_load_\w+[^\n]*\blds\b", txt), src
    assert seen > 0


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="ROCm llvm-objdump absent")
def test_product_has_no_unclear_dma_address_reuse():
    """tools/dma_hazard_scan.py over the product objects: no ds_read takes
    the address registers of an in-flight LDS-DMA of a form the probe did not
    clear (only the 64-bit vaddr form is in the library, and its reuse sites
    are cleared by tools/dma_war_probe.hip, profiles/r05_dma_war_probe.json;
    the GPU side re-runs the probe: tests/test_gpu_dma_probe.py)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import dma_hazard_scan as S
    findings, cleared = [], []
    dma_sites = 0
    for obj in S.product_objects():
        text = S.disassemble(obj, require=False)
        dma_sites += text.count("global_load_lds")
        f, c = S.classify(S.scan(text))
        findings += f
        cleared += c
    # the scan saw the product's LDS-DMA code at all (an empty disassembly
    # would otherwise pass vacuously)
    assert dma_sites > 100, dma_sites
    assert not findings, findings[:5]
    assert all(S.dma_form(h[1]) == "vaddr64" for h in cleared), [h for h in cleared if S.dma_form(h[1]) != "vaddr64"][:5]


def test_dma_scanner_flags_the_probe_patterns():
    """The scanner itself: on the probe kernel's code (every DMA form followed
    by a ds_read into its address registers) it must report the SADDR and
    MUBUF sites as findings and the vaddr sites as cleared."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    import dma_hazard_scan as S
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc absent")
    d = tempfile.mkdtemp()
    try:
        out = os.path.join(d, "probe.s")
        subprocess.run([hipcc, "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        os.path.join(root, "tools", "dma_war_probe.hip"), "-o", out], check=True, capture_output=True)
        findings, cleared = S.classify(S.scan(open(out).read()))
    finally:
        shutil.rmtree(d)
    assert {S.dma_form(h[1]) for h in findings} == {"saddr", "mubuf"}, findings
    assert len(cleared) >= 4 and {S.dma_form(h[1]) for h in cleared} == {"vaddr64"}

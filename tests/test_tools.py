"""CPU checks of the measurement tools: every tools/ablate.py variant still
applies to the product sources (a pattern that no longer matches would make
an A/B silently time the unmodified kernel), and tools/dma_hazard_scan.py
flags an LDS-DMA whose address register a ds_read overwrites."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import ablate  # noqa: E402
import dma_hazard_scan  # noqa: E402
from monocular_depth_estimation_trt_amd import _build  # noqa: E402


def test_ablation_patterns_match_the_sources():
    for name, (fname, subs) in ablate.VARIANTS.items():
        with open(os.path.join(_build.CSRC, fname)) as f:
            src = f.read()
        for old, _new, count in subs:
            assert src.count(old) == count, (name, old[:60])


def test_dma_hazard_scan_flags_lds_return_into_dma_address():
    asm = """
_Zkernel:
\tbuffer_load_dwordx4 v145, s[12:15], 0 offen lds
\tv_add_u32_e32 v168, v160, v209
\tds_read_b128 v[144:147], v168
\ts_endpgm
_Zother:
\tglobal_load_lds_dwordx4 v[4:5], off
\tv_add_u32_e32 v4, 64, v4
\tds_read_b128 v[2:5], v6
\ts_endpgm
"""
    hits = dma_hazard_scan.scan(asm)
    # the first kernel's ds_read overwrites v145; in the second a VALU write
    # (interlocked) comes first and ends the window
    assert [h[0] for h in hits] == ["_Zkernel"]

"""Static instruction census of the attention kernel's hot loop (CPU only:
hipcc cross-compiles gfx950 here).  Guards the VALU budget per MFMA that the
r02 verdict set for the B = 48 kernel (attn_fwd_kernel<8, false, 2, 1, 1>):
the softmax of one 32-key block -- 8 row-max, 16 exp2, 8 f16 packs, 16
row-sum adds -- against its 8 v_mfma_f32_32x32x16_f16 (4 for S^T = K Q^T, 4
for O^T += V^T P^T), i.e. <= 6.5 VALU and exactly 2 transcendentals per
MFMA on the path taken when no running max moves and no key is masked
(tools/isa_census.py; profiles/r03_v1_attn_isa_census.json)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")), reason="hipcc absent")
def test_attention_hot_loop_valu_per_mfma():
    import isa_census
    dis = isa_census.disassemble(os.path.join(ROOT, "monocular_depth_estimation_trt_amd", "csrc", "attention.hip"))
    ks = isa_census.kernels(dis)
    name = next(k for k in ks if "attn_fwd_kernelILi8ELb0ELi2ELi1ELi1EE" in k)
    res = isa_census.analyse(ks[name])
    hot = res["hot_path"]
    assert hot["classes"]["mfma"] % 8 == 0 and hot["classes"]["mfma"] >= 16, hot
    assert hot["valu_per_mfma"] <= 6.5, hot
    assert hot["trans_per_mfma"] == 2.0, hot  # exactly the 16 exp2 per 8 MFMAs


@pytest.mark.skipif(not (shutil.which("hipcc") or os.path.exists("/opt/rocm/bin/hipcc")), reason="hipcc absent")
def test_attention16_hot_loop_census():
    """The default B = 48 kernel since round 6 (attn16_fwd_kernel<8, 1>, switch
    "attn16"): per 32-key block 18 v_mfma_f32_16x16x32_f16 (8 score, 8 P.V,
    2 row sums against an all-ones operand) and the softmax's 16 exp2 -- 8/9
    transcendental per MFMA -- with no fp32 row-sum adds left; the census
    region's VALU (softmax, LDS addressing, the loop's rare rescale and
    masking paths) at <= 3 per MFMA (2.81 measured; the 32x32x16 kernel's
    6.28 per MFMA of twice the work is 3.14 per 16-cycle unit)."""
    import isa_census
    dis = isa_census.disassemble(os.path.join(ROOT, "monocular_depth_estimation_trt_amd", "csrc", "attention.hip"))
    ks = isa_census.kernels(dis)
    name = next(k for k in ks if "attn16_fwd_kernelILi8ELi1EE" in k)
    hot = isa_census.analyse(ks[name])["hot_path"]
    assert hot["classes"]["mfma"] % 18 == 0 and hot["classes"]["mfma"] >= 36, hot
    assert hot["valu_per_mfma"] <= 3.0, hot
    assert 0.85 <= hot["trans_per_mfma"] <= 0.95, hot
    assert hot["valu_by_mnemonic"].get("v_add_f32_e32", 0) <= 2, hot  # the row sums are on the matrix core

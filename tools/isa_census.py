"""Instruction census of a gfx950 kernel's main loop.

    python tools/isa_census.py [--kernel SUBSTR] [--src csrc/attention.hip] [--json out.json]

Compiles the source device-only for gfx950 with the product flags
(`_build.FLAGS` + `_build.PER_FILE`), disassembles it, picks the kernel whose
mangled name contains SUBSTR, finds its loops (a branch back to an earlier
address) and, for the largest loop body, counts the instructions by class:
MFMA, transcendental VALU (v_exp/v_log/v_rcp/...), other VALU by mnemonic,
LDS, VMEM, SALU, branches, waits.  "VALU per MFMA" is the figure the r02
verdict asks for; the straight-line instruction count of the body is a static
census (branches taken rarely, e.g. the online-softmax rescale, are listed
separately from the always-executed part when the body has an inner branch).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def disassemble(src: str) -> str:
    from monocular_depth_estimation_trt_amd import _build
    name = os.path.basename(src)
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "dev.o")
        cmd = [_build.hipcc(), *_build.FLAGS, *_build.PER_FILE.get(name, []), "--cuda-device-only",
               "--no-gpu-bundle-output", "-c", src, "-o", obj]
        subprocess.run(cmd, check=True, capture_output=True)
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", obj], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis: str):
    cur, out = None, {}
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            out[cur] = []
            continue
        m = re.match(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):(.*)$", line)
        if cur and m:
            # operands + the trailing <kernel+0xoff> branch-target annotation
            out[cur].append((int(m.group(3), 16), m.group(1), (m.group(2) + m.group(4)).strip()))
    return out


def classify(mn: str) -> str:
    if mn.startswith("v_mfma"):
        return "mfma"
    if mn.startswith(TRANS):
        return "valu_trans"
    if mn.startswith(("v_accvgpr_",)):
        return "valu_accmov"
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith("s_cbranch") or mn == "s_branch":
        return "branch"
    if mn.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_setprio")):
        return "wait_sync"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def census(insts):
    cls = collections.Counter(classify(mn) for _, mn, _ in insts)
    valu = collections.Counter(mn for _, mn, _ in insts if classify(mn).startswith("valu"))
    return cls, valu


def analyse(insts):
    """Census dict of one kernel's instruction list (kernels()[name])."""
    addr_idx = {ad: i for i, (ad, _, _) in enumerate(insts)}
    # loops: backward branches (objdump prints the target as <kernel+0xoff>)
    loops = []
    for i, (ad, mn, ops) in enumerate(insts):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            m = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", ops)
            if m:
                j = addr_idx.get(insts[0][0] + int(m.group(1), 16))
                if j is not None and j < i:
                    loops.append((i - j, j, i))
    loops.sort(reverse=True)
    res = {"total_insts": len(insts)}
    tot_cls, _ = census(insts)
    res["kernel_classes"] = dict(tot_cls)
    if not loops:
        return res
    n, j, i = loops[0]
    body = insts[j:i + 1]
    cls, valu = census(body)
    # forward branches inside the body: the skipped ranges are conditional code
    cond = []
    for k, (ad, mn, ops) in enumerate(body):
        if mn.startswith("s_cbranch"):
            m = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", ops)
            if m:
                tgt = insts[0][0] + int(m.group(1), 16)
                if ad < tgt <= body[-1][0]:
                    kk = next(x for x in range(k, len(body)) if body[x][0] >= tgt)
                    cond.append({"from": hex(ad), "to": hex(tgt), "insts": kk - k - 1,
                                 "classes": dict(census(body[k + 1:kk])[0])})
    nm = cls["mfma"]
    v_all = cls["valu"] + cls["valu_trans"] + cls["valu_accmov"]
    res["loop"] = {"insts": len(body), "start": hex(body[0][0]), "end": hex(body[-1][0]),
                   "classes": dict(cls), "valu_by_mnemonic": dict(valu.most_common()),
                   "valu_per_mfma_static": round(v_all / nm, 2) if nm else None,
                   "conditional_ranges": cond}
    # hot path: the loop body minus the forward-skipped ranges that hold no
    # MFMA -- the last-block key mask and the online-softmax rescale, taken
    # on a few blocks per row (ranges WITH MFMAs, e.g. "wave active", run)
    skip = set()
    for c in cond:
        if c["classes"].get("mfma", 0) == 0:
            lo, hi = int(c["from"], 16), int(c["to"], 16)
            skip.update(k for k, (ad, _, _) in enumerate(body) if lo < ad < hi)
    # the first branch back to the loop head closes the hot iteration (the
    # code after it, up to the final back-edge, is a rare tail: the last
    # block's rescale falls through there)
    head = body[0][0]
    first_back = len(body) - 1
    for k, (ad, mn, ops) in enumerate(body):
        if mn.startswith("s_cbranch") or mn == "s_branch":
            m = re.search(r"<[^+>]+\+0x([0-9a-f]+)>", ops)
            if m and insts[0][0] + int(m.group(1), 16) == head:
                first_back = k
                break
    hot = [x for k, x in enumerate(body) if k not in skip and k <= first_back]
    hcls, hvalu = census(hot)
    hv = hcls["valu"] + hcls["valu_trans"] + hcls["valu_accmov"]
    if nm:
        res["hot_path"] = {"insts": len(hot), "classes": dict(hcls), "valu_by_mnemonic": dict(hvalu.most_common()),
                           "valu_per_mfma": round(hv / nm, 2),
                           "trans_per_mfma": round(hcls["valu_trans"] / nm, 2),
                           "salu_per_mfma": round(hcls["salu"] / nm, 2)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "monocular_depth_estimation_trt_amd", "csrc", "attention.hip"))
    ap.add_argument("--kernel", default="attn_fwd_kernelILi8ELb0ELi2ELi1ELi1EE")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    ks = kernels(disassemble(a.src))
    name = next(k for k in ks if a.kernel in k)
    res = {"kernel": name, **analyse(ks[name])}
    out = json.dumps(res, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(out + "\n")
    print(out)


if __name__ == "__main__":
    main()

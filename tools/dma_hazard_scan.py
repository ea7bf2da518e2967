"""Scan gfx950 device code for LDS-DMA address-register reuse.

An LDS-DMA instruction (global_load_lds_* / buffer_load_* ... lds) whose
address VGPRs are next written by a ds_read (an asynchronous LDS return)
before the DMA's vmcnt wait is the pattern round 4's fused-MLP experiment
was suspected of (nondeterministic outputs).  This
scanner lists, per kernel, every such site within WINDOW instructions of the
DMA; VALU overwrites right after a VMEM issue are in every compiled kernel
and are not listed.

The rule it checks (round 5): the hardware reads an LDS-DMA's address VGPRs
when the instruction issues, so a later ds_read may take those registers.
Measured on MI355X by tools/dma_war_probe.hip
(profiles/r05_dma_war_probe.json): 1.68e11 lane-DMAs per form with a
ds_read overwriting the address registers as the very next instruction
(4 DMAs in flight per wave, 8 x 4 waves per CU, 1 GiB source so the TA
queues stay full) returned 0 wrong rows for the 64-bit vaddr form, the
SADDR form and the MUBUF `offen lds` form alike, while the positive control
(decoy address in the registers before the issue) returned the decoy on every
lane.  The product keeps the 64-bit vaddr form anyway except in the panel
GEMM (SADDR form, no reuse site allowed; tests/test_lds_dma_form.py);
a reuse site behind any OTHER form is reported as a finding (exit 1), the
vaddr-form sites as cleared by the probe (listed with --list).

    python tools/dma_hazard_scan.py [--list] file.s|file.o [...]
    python tools/dma_hazard_scan.py --product [--list]   (the in-tree build's objects)
"""
from __future__ import annotations

import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

WINDOW = 24
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_FN_S = re.compile(r"^(_Z\S*):")                       # hipcc -S label
_FN_D = re.compile(r"^[0-9a-f]+ <(_Z\S*)>:")           # llvm-objdump -d label


def _regs(tok: str) -> set[int]:
    out: set[int] = set()
    for m in _VREG.finditer(tok):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _dest(line: str) -> set[int]:
    """VGPRs an instruction writes (first operand of a VALU / DS read / VMEM
    load; stores, DMA, MFMA-to-AGPR and scalar ops write none)."""
    parts = line.split(None, 1)
    if len(parts) < 2:
        return set()
    op, args = parts[0], parts[1]
    if op.startswith(("s_", "ds_write", "global_store", "buffer_store", "flat_store", "scratch_store")):
        return set()
    if "lds" in args.split() or op.startswith("global_load_lds"):
        return set()
    first = args.split(",")[0]
    return _regs(first) if first.strip().startswith("v") else set()


def dma_form(line: str) -> str | None:
    """'vaddr64' (global_load_lds v[a:b], off), 'saddr' (v, s[..]), 'mubuf'
    (buffer_load ... lds), or None for any other instruction."""
    parts = line.split(None, 1)
    if len(parts) < 2:
        return None
    op, args = parts[0], parts[1]
    if op.startswith("global_load_lds"):
        return "saddr" if re.search(r",\s*s\[", args) else "vaddr64"
    if op.startswith("buffer_load") and re.search(r"\blds\b", args):
        return "mubuf"
    return None


def _dma_addr(line: str) -> set[int] | None:
    if dma_form(line) is None:
        return None
    return _regs(line.split(None, 1)[1].split(",")[0])


def scan(asm: str) -> list[tuple[str, str, str]]:
    """(kernel, DMA line, overwriting ds_read line) for every reuse site."""
    hits = []
    fn = "?"
    code = []
    for raw in asm.splitlines():
        l = raw.split("//")[0].strip()
        m = _FN_S.match(l) or _FN_D.match(l)
        if m:
            fn = m.group(1)
            continue
        if not l or l.startswith((";", ".")) or l.endswith(":"):
            continue
        code.append((fn, l))
    for i, (fn, l) in enumerate(code):
        addr = _dma_addr(l)
        if not addr:
            continue
        for fn2, l2 in code[i + 1:i + 1 + WINDOW]:
            if fn2 != fn:
                break
            if _dma_addr(l2) is not None:
                continue  # a later DMA reusing the register reads it the same way
            d = _dest(l2)
            if d & addr:
                if l2.split()[0].startswith("ds_read"):
                    hits.append((fn, l, l2))
                break
    return hits


def classify(hits):
    """(findings, cleared): reuse sites behind a non-vaddr DMA form are
    findings; vaddr64 sites are cleared by the probe (module docstring)."""
    findings = [h for h in hits if dma_form(h[1]) != "vaddr64"]
    cleared = [h for h in hits if dma_form(h[1]) == "vaddr64"]
    return findings, cleared


def disassemble(obj: str, require: bool = True) -> str:
    """Device (gfx950) disassembly of a hipcc object or shared library;
    `require=False` for objects that may hold host code only (engine.hip)."""
    d = tempfile.mkdtemp()
    try:
        c = os.path.join(d, os.path.basename(obj))
        shutil.copy(obj, c)
        subprocess.run([OBJDUMP, "--offloading", c], capture_output=True, check=True)
        dev = [f for f in glob.glob(c + ".*") if f.endswith("gfx950")]
        if not dev and not require:
            return ""
        if not dev:
            # a silent "" would let a caller scan nothing and report clean
            # (e.g. after an MDE_OFFLOAD_ARCH or llvm-objdump naming change)
            raise RuntimeError(f"{obj}: no gfx950 device bundle found by {OBJDUMP} --offloading")
        return subprocess.run([OBJDUMP, "-d", dev[0]], capture_output=True, text=True, check=True).stdout
    finally:
        shutil.rmtree(d)


def product_objects() -> list[str]:
    sys.path.insert(0, ROOT)
    from monocular_depth_estimation_trt_amd import _build
    _build.build_library(verbose=False)
    return [os.path.join(_build.OBJDIR, s + ".o") for s in _build.SOURCES]


def main(argv: list[str]) -> int:
    files = [a for a in argv if not a.startswith("--")]
    if "--product" in argv:
        files += product_objects()
    total_f = total_c = dma = 0
    for f in files:
        text = open(f).read() if f.endswith(".s") else disassemble(f, require="--product" not in argv)
        dma += text.count("global_load_lds") + text.count(" lds\n")
        findings, cleared = classify(scan(text))
        total_f += len(findings)
        total_c += len(cleared)
        print(f"{os.path.basename(f)}: {len(findings)} finding(s), {len(cleared)} vaddr64 reuse(s) cleared by the probe "
              f"in {len({h[0] for h in cleared})} kernel(s)")
        show = findings + (cleared if "--list" in argv else [])
        for k in sorted({h[0] for h in show})[:40]:
            ex = next(h for h in show if h[0] == k)
            print(f"   {k[:90]}\n      {ex[1]}\n      -> {ex[2]}")
    print(f"total: {total_f} finding(s), {total_c} cleared site(s), {dma} LDS-DMA instruction(s) scanned")
    if files and not dma:
        print("error: no LDS-DMA instruction in the scanned device code (nothing was checked)")
        return 2
    return 1 if total_f else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

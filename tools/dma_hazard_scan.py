"""Scan gfx950 assembly for LDS-DMA address-register reuse.

An LDS-DMA instruction (global_load_lds_* / buffer_load_* ... lds) whose
address VGPRs are overwritten by a following instruction before the DMA has
read them corrupted the fused MLP's weight ring (round 4: nondeterministic
outputs until the address registers were kept live).  This scanner lists,
per kernel, every DMA whose address VGPR is next written by a ds_read
(asynchronous LDS return) within WINDOW instructions; VALU overwrites right
after the DMA are common in every deterministic kernel and are not flagged.

    python tools/dma_hazard_scan.py file.s [file.s ...]
    python tools/dma_hazard_scan.py --build      (hipcc -S every csrc/*.hip)
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

WINDOW = 24
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "monocular_depth_estimation_trt_amd", "csrc")

_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


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


def _dma_addr(line: str) -> set[int] | None:
    parts = line.split(None, 1)
    if len(parts) < 2:
        return None
    op, args = parts[0], parts[1]
    if op.startswith("global_load_lds"):
        return _regs(args.split(",")[0])
    if op.startswith("buffer_load") and re.search(r"\blds\b", args):
        return _regs(args.split(",")[0])
    return None


def scan(asm: str) -> list[tuple[str, str, str]]:
    hits = []
    fn = "?"
    lines = [l.strip() for l in asm.splitlines()]
    code = []
    for l in lines:
        if re.match(r"^_Z\S*:", l):
            fn = l.split(":")[0]
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
                break  # a VALU overwrite is interlocked (every product kernel does it); an LDS return is not
    return hits


def main(argv: list[str]) -> int:
    files = [a for a in argv if not a.startswith("--")]
    if "--build" in argv:
        tmp = tempfile.mkdtemp()
        for src in sorted(os.listdir(CSRC)):
            if src.endswith(".hip"):
                out = os.path.join(tmp, src + ".s")
                subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                                "--cuda-device-only", "-S", os.path.join(CSRC, src), "-o", out],
                               check=True, capture_output=True)
                files.append(out)
    total = 0
    for f in files:
        with open(f) as fh:
            hits = scan(fh.read())
        total += len(hits)
        kern = sorted({h[0] for h in hits})
        print(f"{os.path.basename(f)}: {len(hits)} reuse(s) in {len(kern)} kernel(s)")
        for k in kern[:20]:
            ex = next(h for h in hits if h[0] == k)
            print(f"   {k[:90]}\n      {ex[1]}\n      -> {ex[2]}")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

"""Per-segment timing of the panel GEMM (gemm_panel.hip built with -DPX_TRACE):
runs one fc1-shaped launch (ViT-S B=48: M 65760, N 1536, K 384, GELU) through
the C ABI with the switch on, reads the s_memtime stamps of blocks 0-7 and
prints, per group and segment kind, the work time and the barrier wait.

    python tools/panel_trace.py LIB [--act 2] [--n 1536]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--act", type=int, default=2)
    ap.add_argument("--n", type=int, default=1536)
    ap.add_argument("--m", type=int, default=65760)
    a = ap.parse_args()
    import torch
    from gpu_util import pad_w, ptr, stream
    from monocular_depth_estimation_trt_amd import _lib
    _lib.use_library(a.lib)
    L = _lib.lib()
    _lib.set_tuning("panel", 1)
    dev = torch.device("cuda:0")
    m, n, k = a.m, a.n, 384
    x = torch.randn(m, k, device=dev).half()
    wp = pad_w(torch.randn(n, k) * k ** -0.5).to(dev)
    b = torch.randn(n, device=dev) * 0.1
    out = torch.empty(m, n, dtype=torch.float16, device=dev)
    for _ in range(3):
        L.mde_op_linear(ptr(x), k, ptr(wp), wp.shape[1], m, n, k, ptr(b), a.act, ptr(out), n, stream())
    torch.cuda.synchronize()
    buf = np.zeros((8, 8, 96, 4), dtype=np.uint64)
    fn = getattr(L, "mde_debug_panel_trace")
    fn.argtypes = [C.c_void_p]
    assert fn(buf.ctypes.data) == 0
    t = buf.astype(np.int64)
    nseg = int((t[0, 0, :90, 0] > 0).sum())
    print(f"units recorded per wave: {nseg}")
    rows = []
    for blk in range(8):
        st, en, wt = t[blk, :, :, 0], t[blk, :, :, 1], t[blk, :, :, 2]
        for u in range(1, nseg - 1):
            length = st[:, u + 1].max() - st[:, u].max()  # barrier to barrier
            work = (en[:, u] - st[:, u]).mean()            # after barrier -> before the end-of-unit wait
            wait = (wt[:, u] - en[:, u]).mean()            # the vmcnt(0)
            skew = (st[:, u + 1] - wt[:, u]).mean()        # waiting at the barrier
            spread = (en[:, u] - st[:, u]).max() - (en[:, u] - st[:, u]).min()
            rows.append((length, work, wait, skew, spread))
    r = np.array(rows, dtype=np.float64)
    print(f"unit (s_memtime ticks, n={len(r)}): length {r[:, 0].mean():7.0f}  work {r[:, 1].mean():7.0f}  "
          f"vmcnt wait {r[:, 2].mean():7.0f}  barrier {r[:, 3].mean():7.0f}  work spread over waves {r[:, 4].mean():7.0f}")

    # in-kernel clock: memtime ticks per 100 MHz realtime tick over each wave's units
    ck = []
    for blk in range(8):
        for w in range(8):
            mt, rt = t[blk, w, :nseg, 0], t[blk, w, :nseg, 3]
            if rt[-1] > rt[0]:
                ck.append((mt[-1] - mt[0]) / (rt[-1] - rt[0]) * 0.1)
    if ck:
        print(f"in-kernel clock {np.median(ck):.3f} GHz (median over waves); units {nseg}, "
              f"first -> last unit start {np.median([(t[b, 0, nseg - 1, 3] - t[b, 0, 0, 3]) / 100.0 for b in range(8)]):.1f} us")
    # whole-kernel phases (panel32 trace builds): realtime stamps, us
    rt = t[:, :, :, 3].astype(np.float64) / 100.0
    if (t[:, :, 95, 3] > 0).all():
        ent, p0, p1, end = rt[:, :, 95], rt[:, :, 91], rt[:, :, 92], rt[:, :, 90]
        u0 = rt[:, :, 0]
        print(f"per wave (median over blocks 0-7, us): entry -> first panel load start {np.median(p0 - ent):.2f}, "
              f"first panel load {np.median(p1 - p0):.2f}, -> first unit {np.median(u0 - p1):.2f}; "
              f"entry -> end {np.median(end - ent):.2f}")
        sw = t[:, :, 93, 3] > 0
        if sw.any():
            print(f"mid-run panel switch (epilogue + A load + stats + drain): "
                  f"{np.median((rt[:, :, 94] - rt[:, :, 93])[sw]):.2f} us over {int(sw.sum())} waves")
        print(f"spread of kernel-entry times over blocks 0-7: {ent[:, 0].max() - ent[:, 0].min():.2f} us; "
              f"of end times {end[:, 0].max() - end[:, 0].min():.2f} us")
    lo = np.array([(t[b, :4, 1:nseg - 1, 1] - t[b, :4, 1:nseg - 1, 0]).mean() for b in range(8)])
    hi = np.array([(t[b, 4:, 1:nseg - 1, 1] - t[b, 4:, 1:nseg - 1, 0]).mean() for b in range(8)])
    print(f"work per unit: waves 0-3 {lo.mean():7.0f}  waves 4-7 {hi.mean():7.0f}")


if __name__ == "__main__":
    main()

"""In-graph clock and unit timing of the panel GEMM (a PX_TRACE build of the
library): replays the bench's ViT-S 518^2 B=48 forward graph back to back, as
bench.py times it, then reads the s_memtime / s_memrealtime stamps the LAST
panel launch of the last forward (block 11's fc1) left for workgroups 0-7.

    python tools/graph_clock.py LIB [--steps 40] [--batch 48]

The standalone trace (tools/panel_trace.py) runs the kernel alone on an idle
chip; inside the graph the chip runs at the clock the whole forward's power
draw allows, which is what a step-time A/B actually sees.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--batch", type=int, default=48)
    a = ap.parse_args()
    import torch
    from monocular_depth_estimation_trt_amd import _lib, pack, weights
    _lib.use_library(a.lib)
    from monocular_depth_estimation_trt_amd.engine import Engine
    L = _lib.lib()
    B, S = a.batch, 518
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    x = torch.from_numpy(weights.synthetic_images(B, S, S, first_seed=100)).to("cuda:0")
    y = torch.empty(B, S, S, device="cuda:0")
    eng = Engine.from_bytes(pack.pack_bytes(sd, cfg, S, S), 0, profile=((1, 3, S, S), (B, 3, S, S), (B, 3, S, S)))
    ctx = eng.create_execution_context()
    ctx.set_input_shape("input", tuple(x.shape))
    ctx.set_tensor_address("input", x.data_ptr())
    ctx.set_tensor_address("output", y.data_ptr())
    st = torch.cuda.Stream()
    for _ in range(5):
        ctx.execute_async_v3(st.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(st):
        e0.record()
        for _ in range(a.steps):
            ctx.execute_async_v3(st.cuda_stream)
        e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    buf = np.zeros((8, 8, 96, 4), dtype=np.uint64)
    fn = getattr(L, "mde_debug_panel_trace")
    fn.argtypes = [C.c_void_p]
    assert fn(buf.ctypes.data) == 0
    t = buf.astype(np.int64)
    nseg = int((t[0, 0, :90, 0] > 0).sum())
    ck = []
    for b in range(8):
        for w in range(8):
            mt, rt = t[b, w, :nseg, 0], t[b, w, :nseg, 3]
            if rt[nseg - 1] > rt[0]:
                ck.append((mt[nseg - 1] - mt[0]) / (rt[nseg - 1] - rt[0]) * 0.1)
    ul = []
    for b in range(8):
        st_ = t[b, :, :nseg, 0]
        ul += list(np.diff(st_.max(0))[1:-1])
    rt = t[:, :, :, 3].astype(np.float64) / 100.0
    print(f"graph step {ms:.3f} ms ({B * 1000 / ms:.1f} img/s); last panel launch: {nseg} units per workgroup, "
          f"in-kernel clock {np.median(ck):.3f} GHz, unit {np.median(ul):.0f} ticks = "
          f"{np.median(ul) / np.median(ck) / 1e3:.2f} us")
    if (t[:, :, 95, 3] > 0).all():
        print(f"entry -> end {np.median(rt[:, :, 90] - rt[:, :, 95]):.1f} us (workgroups 0-7)")
    ctx.destroy()
    eng.destroy()


if __name__ == "__main__":
    main()

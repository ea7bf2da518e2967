"""Time the hot-path kernels at DA-V2 shapes (rank-0 tuning aid, GPU box).

    python tools/bench_kernels.py [--batch 32] [--lib path/to/libmde_hip.so]

Each op is launched through the C ABI on torch's current stream and timed
with torch.cuda.Event over `--iters` back-to-back launches (after warmup).
TF/s uses the algorithmic FLOP of that launch.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default="")
    ap.add_argument("--only", default="")
    ap.add_argument("--attn-cfgs", default="", help="comma list of attention launch configs to time (mde_op_attention_cfg)")
    ap.add_argument("--dim", type=int, default=384, help="ViT width D (ViT-L: 1024)")
    ap.add_argument("--heads", type=int, default=6, help="attention heads (ViT-L: 16)")
    ap.add_argument("--tokens", type=int, default=1370, help="tokens per image (GEMM rows = batch x tokens)")
    ap.add_argument("--cold", action="store_true",
                    help="also time each launch alone after a 512 MB write (caches cold, as in the graph)")
    a = ap.parse_args()
    import torch
    from gpu_util import conv_w, pad_w, ptr, stream
    from monocular_depth_estimation_trt_amd import _lib
    if a.lib:
        _lib.use_library(a.lib)
    dev = torch.device("cuda:0")
    B, T, D, H = a.batch, a.tokens, a.dim, a.heads
    M = B * T
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s, scale=1.0, dtype=torch.float16):
        return (torch.randn(*s, generator=g, device=dev) * scale).to(dtype)

    def timeit(name, fn, flop):
        if a.only and a.only not in name:
            return
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        line = f"{name:28s} {ms * 1e3:9.1f} us  {flop / ms / 1e9:8.1f} TF/s"
        if a.cold:
            cold = []
            for _ in range(max(5, a.iters // 4)):
                flush.fill_(1.0)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                cold.append(e0.elapsed_time(e1))
            cms = sorted(cold)[len(cold) // 2]
            line += f"   cold {cms * 1e3:9.1f} us  {flop / cms / 1e9:8.1f} TF/s"
        print(line, flush=True)

    L = _lib.lib()
    st = stream()
    flush = torch.empty(128 << 20, device=dev) if a.cold else None  # 512 MB > L2 + Infinity Cache
    x16 = rnd(M, 4 * D)
    out = torch.empty(M, 4 * D, dtype=torch.float16, device=dev)
    x32 = torch.randn(M, D, device=dev)
    bias = torch.randn(4 * D, device=dev) * 0.02
    ls = torch.full((4 * D,), 0.5, device=dev)
    for name, n, k, act in ((f"qkv-like N{3 * D} K{D}", 3 * D, D, 0), (f"fc1 N{4 * D} K{D} gelu", 4 * D, D, 2),
                            (f"fc1 N{4 * D} K{D} nogelu", 4 * D, D, 0)):
        w = pad_w(rnd(n, k, scale=k ** -0.5))
        timeit(name, lambda: L.mde_op_linear(ptr(x16), k, ptr(w), w.shape[1], M, n, k, ptr(bias), act, ptr(out),
                                             n, st), 2.0 * M * n * k)
    for name, n, k in ((f"proj N{D} K{D} resid", D, D), (f"fc2 N{D} K{4 * D} resid", D, 4 * D)):
        w = pad_w(rnd(n, k, scale=k ** -0.5))
        timeit(name, lambda: L.mde_op_linear_residual(ptr(x16), k, ptr(w), w.shape[1], M, n, k, ptr(bias), ptr(ls),
                                                      ptr(x32), D, st), 2.0 * M * n * k)
    Tp = (T + 63) // 64 * 64
    w = pad_w(rnd(3 * D, D, scale=D ** -0.5))
    q = torch.zeros(B * H, Tp, 64, dtype=torch.float16, device=dev)
    k_ = torch.zeros_like(q)
    vt = torch.zeros(B * H, 64, Tp, dtype=torch.float16, device=dev)
    timeit(f"qkv N{3 * D} K{D} (E_QKV)", lambda: L.mde_op_qkv(ptr(x16), ptr(w), w.shape[1], ptr(bias), B, T, H, Tp,
                                                        0.125, ptr(q), ptr(k_), ptr(vt), st), 2.0 * M * 3 * D * D)
    # the engine's operands: q pre-scaled by dh^-0.5 * log2(e) (E_QKV), so
    # scores are O(1) in log2 units -- unscaled N(0,1) q and k would put the
    # score std at 8 and fire the online-softmax rescale on most blocks
    q.normal_().mul_(0.125 * 1.4426950408889634 * float(os.environ.get("ATTN_QSCALE", "1")))
    k_.normal_()
    vt.normal_()
    o = torch.empty(M, D, dtype=torch.float16, device=dev)
    timeit(f"attention T{T} H{H}", lambda: L.mde_op_attention(ptr(q), ptr(k_), ptr(vt), ptr(o), B, H, T, Tp, D, st),
           4.0 * B * H * T * T * 64)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
    for cfg in [c for c in a.attn_cfgs.replace("+", ",").split(",") if c]:
        timeit(f"attention T{T} H{H} cfg {cfg}",
               lambda: L.mde_op_attention_cfg(ptr(q), ptr(k_), ptr(vt), ptr(o), B, H, T, Tp, D, cfg.encode(), ptr(ws),
                                              ws.numel(), st), 4.0 * B * H * T * T * 64)
    F = 64
    for hw in (148, 74):
        xin = rnd(B, hw, hw, F)
        w = conv_w(rnd(F, F, 3, 3, scale=(9 * F) ** -0.5).float())
        oc = torch.empty(B, hw, hw, F, dtype=torch.float16, device=dev)
        timeit(f"rcu conv3x3 {hw}^2 64->64", lambda: L.mde_op_conv3x3(ptr(xin), B, hw, hw, F, ptr(w), w.shape[1], F,
                                                                    1, 1, ptr(bias), 1, ptr(None), ptr(None),
                                                                    ptr(oc), st), 2.0 * B * hw * hw * F * F * 9)
    xin = rnd(B, 148, 148, F)
    w = conv_w(rnd(32, F, 3, 3, scale=(9 * F) ** -0.5).float())
    oc = torch.empty(B, 296, 296, 32, dtype=torch.float16, device=dev)
    timeit("head conv1 up148->296 64->32", lambda: L.mde_op_conv3x3_up(ptr(xin), B, 148, 148, F, 296, 296, ptr(w),
                                                                       w.shape[1], 32, ptr(bias), 0, ptr(oc), st),
           2.0 * B * 296 * 296 * 32 * F * 9)
    xin = rnd(B, 296, 296, 32)
    w = conv_w(rnd(32, 32, 3, 3, scale=(9 * 32) ** -0.5).float())
    w2 = torch.randn(32, device=dev) * 0.2
    od = torch.empty(B, 518, 518, device=dev)
    timeit("head conv2 up296->518 +1x1", lambda: L.mde_op_depth_head(ptr(xin), B, 296, 296, 32, 518, 518, ptr(w),
                                                                     w.shape[1], ptr(bias), ptr(w2), 0.1, 1, 20.0,
                                                                     ptr(od), st), 2.0 * B * 518 * 518 * 32 * 32 * 9)


if __name__ == "__main__":
    main()

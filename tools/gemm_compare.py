"""hipBLASLt (torch.nn.functional.linear) vs the library GEMM (mde_op_linear,
plain store epilogue) at the dense shapes of a workload.  GPU box tuning aid.

    python tools/gemm_compare.py [--set depth_pro|vits32|vitl8] [--iters 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SETS = {
    # Depth Pro patch encoder at B=4: 140 sequences x 577 tokens, D 1024
    "depth_pro": [(80780, 3072, 1024), (80780, 1024, 1024), (80780, 4096, 1024), (80780, 1024, 4096)],
    # DA-V2 ViT-S at B=32
    "vits32": [(43840, 1152, 384), (43840, 384, 384), (43840, 1536, 384), (43840, 384, 1536)],
    # DA-V2 ViT-L at B=8
    "vitl8": [(10960, 3072, 1024), (10960, 1024, 1024), (10960, 4096, 1024), (10960, 1024, 4096)],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="depth_pro", choices=sorted(SETS))
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    import torch
    from gpu_util import ptr, stream
    from monocular_depth_estimation_trt_amd import _lib
    dev = torch.device("cuda:0")

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    _lib.lib()
    for M, N, K in SETS[a.set]:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        w = torch.randn(N, K, device=dev, dtype=torch.float16) * K ** -0.5
        wp = torch.zeros((N + 127) // 128 * 128, (K + 63) // 64 * 64, device=dev, dtype=torch.float16)
        wp[:N, :K] = w
        out = torch.empty(M, N, device=dev, dtype=torch.float16)
        st = stream()
        ms_t = timeit(lambda: torch.nn.functional.linear(x, w))
        ms_m = timeit(lambda: _lib.call("mde_op_linear", ptr(x), K, ptr(wp), wp.shape[1], M, N, K, ptr(None), 0,
                                        ptr(out), N, st))
        fl = 2.0 * M * N * K
        ref = torch.nn.functional.linear(x[:256], w)
        err = float((out[:256].float() - ref.float()).abs().max())
        print(f"M{M} N{N} K{K}: hipBLASLt {ms_t * 1e3:8.1f} us {fl / ms_t / 1e9:7.1f} TF/s | "
              f"mde {ms_m * 1e3:8.1f} us {fl / ms_m / 1e9:7.1f} TF/s  (max_abs {err:.3e})", flush=True)


if __name__ == "__main__":
    main()

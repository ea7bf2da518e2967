"""Where do the batch-1 GEMMs lose time to cold weights?  GPU box tuning aid.

Times one library GEMM (mde_op_linear, plain store epilogue) at the ViT-L
batch-1 shapes (1370 tokens) in three cache states, events around the GEMM
alone, each state re-made before every timed launch:
  warm   the same GEMM just ran (weights in L2 and the Infinity Cache)
  cold   a 1 GiB buffer written first (L2 and the Infinity Cache flushed)
  mall   flushed, then the weights read once and 64 MiB of other data read
         after them (the weights left in the Infinity Cache, not in L2) --
         the state a side-stream prefetch of the next layer's weights leaves

    python tools/prefetch_probe.py [--reps 20] [--tokens 1370]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

SHAPES = (("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=1370)
    a = ap.parse_args()
    import torch
    from gpu_util import ptr, stream
    from monocular_depth_estimation_trt_amd import _lib
    dev = torch.device("cuda:0")
    _lib.lib()
    flush = torch.empty(1 << 28, device=dev, dtype=torch.float32)     # 1 GiB
    other = torch.empty(1 << 24, device=dev, dtype=torch.float32)     # 64 MiB
    M = a.tokens
    st = stream()
    for name, N, K in SHAPES:
        x = torch.randn(M, K, device=dev, dtype=torch.float16)
        wp = torch.randn((N + 127) // 128 * 128, K, device=dev, dtype=torch.float16) * K ** -0.5
        out = torch.empty(M, N, device=dev, dtype=torch.float16)

        def gemm():
            _lib.call("mde_op_linear", ptr(x), K, ptr(wp), wp.shape[1], M, N, K, ptr(None), 0, ptr(out), N, st)

        res = {}
        for state in ("warm", "cold", "mall"):
            tot = 0.0
            for r in range(a.reps + 2):
                if state == "warm":
                    gemm()
                else:
                    flush.fill_(float(r))
                    if state == "mall":
                        s = wp.float().sum()          # weights through the caches
                        s += other.sum()              # then 64 MiB of other lines
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gemm()
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    tot += e0.elapsed_time(e1)
            res[state] = tot / a.reps * 1e3
        fl = 2.0 * M * N * K
        print(f"{name:5s} M{M} N{N} K{K}: " + "  ".join(f"{s} {us:6.1f} us ({fl / us / 1e6:5.0f} TF/s)"
                                                       for s, us in res.items()), flush=True)


if __name__ == "__main__":
    main()

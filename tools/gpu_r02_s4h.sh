#!/bin/bash
# BK32 / 3-stage / 3-per-CU 128^2 GEMM with half-size epilogue staging: parity, then same-box A/B at B=28 and ViT-L B=8
set -o pipefail
o=gpurun_out/s4h; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread > $o/ops.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $o/engine.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/bk32_$r.json 2> $o/bk32_$r.err || exit $?
  MDE_GEMM_BK32=0 timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/bk64_$r.json 2> $o/bk64_$r.err || exit $?
done
timeout -k 10 300 python -u bench.py --encoder vitl --batch 8 --no-b1 --no-cpu-baseline > $o/vitl_b8_bk32.json 2> $o/vitl_b8_bk32.err || exit $?
MDE_GEMM_BK32=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 8 --no-b1 --no-cpu-baseline > $o/vitl_b8_bk64.json 2> $o/vitl_b8_bk64.err || exit $?

#!/bin/bash
# attention with two 32-query sub-tiles per wave (MDE_ATTN_CFG=8q2, 228 VGPRs, one workgroup per CU): parity + timing
set -o pipefail
o=gpurun_out/s4y; mkdir -p $o
MDE_ATTN_CFG=8q2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k attention -x -q --timeout 120 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for c in 8 8q2 8 8q2; do
  echo "== $c" >> $o/attn.log
  MDE_ATTN_CFG=$c timeout -k 10 120 python tools/bench_kernels.py --batch 28 --only attention --iters 50 >> $o/attn.log 2>&1 || exit $?
done
for c in 8 8q2; do
  MDE_ATTN_CFG=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-b1 > $o/bench_$c.json 2> $o/bench_$c.err || exit $?
done

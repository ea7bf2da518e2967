#!/bin/bash
# attention workgroup shape at the B=48 default: 8 waves x 32 queries vs 4 waves x 32 queries
set -o pipefail
o=gpurun_out/s4ah; mkdir -p $o
for c in 8 4 8 4; do
  echo "== $c" >> $o/attn.log
  MDE_ATTN_CFG=$c timeout -k 10 120 python tools/bench_kernels.py --batch 48 --only attention --iters 40 >> $o/attn.log 2>&1 || exit $?
done
for c in 8 4; do
  MDE_ATTN_CFG=$c timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/bench_$c.json 2> $o/bench_$c.err || exit $?
done

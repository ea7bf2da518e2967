#!/bin/bash
# BK 32 tiles with a 2-stage ring (33 KB, four workgroups per CU) vs 3 stages: same-box A/B at B=28
set -o pipefail
o=gpurun_out/s4r; mkdir -p $o
MDE_LIB=build/var/lib_bk32s2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "linear or qkv" -x -q --timeout 120 --timeout-method thread > $o/ops.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/s3_$r.json 2> $o/s3_$r.err || exit $?
  MDE_LIB=build/var/lib_bk32s2.so timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/s2_$r.json 2> $o/s2_$r.err || exit $?
done

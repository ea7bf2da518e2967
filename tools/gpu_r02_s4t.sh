#!/bin/bash
# residual-update GEMMs (proj K=384, fc2 K=1536) on 128x64 tiles: parity + same-box A/B at B=28
set -o pipefail
o=gpurun_out/s4t; mkdir -p $o
MDE_RESID_N64_KMAX=4096 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -k "residual or 518 or lnfold" -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/base_$r.json 2> $o/base_$r.err || exit $?
  MDE_RESID_N64_KMAX=384 timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/k384_$r.json 2> $o/k384_$r.err || exit $?
  MDE_RESID_N64_KMAX=4096 timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/k4096_$r.json 2> $o/k4096_$r.err || exit $?
done

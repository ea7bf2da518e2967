#!/bin/bash
# direct conv 16x16-pixel tiles on 8 waves (MDE_CONV_TH16=1) for the 64-wide convs: parity + same-box A/B
set -o pipefail
o=gpurun_out/s4aa; mkdir -p $o
MDE_CONV_TH16=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -k "conv or 518 or consistency" -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/base_$r.json 2> $o/base_$r.err || exit $?
  MDE_CONV_TH16=1 timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/th16_$r.json 2> $o/th16_$r.err || exit $?
done
MDE_CONV_TH16=1 timeout -k 10 300 python -u bench.py --batch 1 --steps 40 --no-b1 --no-cpu-baseline > $o/th16_b1.json 2> $o/th16_b1.err || exit $?
timeout -k 10 300 python -u bench.py --batch 1 --steps 40 --no-b1 --no-cpu-baseline > $o/base_b1.json 2> $o/base_b1.err || exit $?

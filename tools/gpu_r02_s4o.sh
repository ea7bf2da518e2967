#!/bin/bash
# 128^2 x 4-slice split-K for the batch-1 ViT-L / VGGT fc2: parity, A/B
set -o pipefail
o=gpurun_out/s4o; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -k "splitk or 518" -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vitl_b1_128_$r.json 2> $o/vitl_b1_128_$r.err || exit $?
  MDE_SPLITK128=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vitl_b1_64_$r.json 2> $o/vitl_b1_64_$r.err || exit $?
done

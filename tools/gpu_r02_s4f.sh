#!/bin/bash
# tuning knobs: 64^2 vs 128^2 tiles for the batch-1 ViT-L GEMMs (MDE_GEMM_BIG_MIN), LDS-resident conv taps (MDE_CONV_BRES)
set -o pipefail
o=gpurun_out/s4f; mkdir -p $o
for v in 240 400 1000; do
  MDE_GEMM_BIG_MIN=$v timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vitl_b1_big$v.json 2> $o/vitl_b1_big$v.err || exit $?
done
for v in 240 1000; do
  MDE_GEMM_BIG_MIN=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vits_b1_big$v.json 2> $o/vits_b1_big$v.err || exit $?
done

#!/bin/bash
# BK32 3-stage tiles for the K=1024 ViT-L stores at batch 1 / 8 (MDE_GEMM_BK32_KMAX)
set -o pipefail
o=gpurun_out/s4j; mkdir -p $o
for b in 1 8; do
  for k in 768 1024; do
    MDE_GEMM_BK32_KMAX=$k timeout -k 10 300 python -u bench.py --encoder vitl --batch $b --steps 20 --no-b1 --no-cpu-baseline > $o/vitl_b${b}_k$k.json 2> $o/vitl_b${b}_k$k.err || exit $?
  done
done

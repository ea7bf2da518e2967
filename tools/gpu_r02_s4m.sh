#!/bin/bash
# direct-conv variants at B=28 and ViT-L B=1: LDS-resident weight taps for CK 64 (bres2), + 32-wide channel tiles (bn32bres2)
set -o pipefail
o=gpurun_out/s4m; mkdir -p $o
for v in base bres2 bn32bres2; do
  lib=monocular_depth_estimation_trt_amd/libmde_hip.so; [ $v != base ] && lib=build/var/lib_$v.so
  MDE_LIB=$lib timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/b28_$v.json 2> $o/b28_$v.err || exit $?
  MDE_LIB=$lib timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline > $o/vitl_b1_$v.json 2> $o/vitl_b1_$v.err || exit $?
done
MDE_LIB=build/var/lib_bn32bres2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv" -x -q --timeout 120 --timeout-method thread > $o/ops.log 2>&1 || exit $?

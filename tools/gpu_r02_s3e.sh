#!/bin/bash
# GEMM latency structure: main-loop-only, 3-stage (1 WG/CU) and BK32x4-stage (2 WG/CU) variants
set -o pipefail
mkdir -p gpurun_out/ab
for v in base bk32 bk32w4; do
  lib=monocular_depth_estimation_trt_amd/libmde_hip.so
  [ $v != base ] && lib=build/var/lib_$v.so
  echo "== $v" >> gpurun_out/ab/gemm.log
  timeout -k 10 120 python tools/bench_kernels.py --lib $lib --batch 28 --iters 30 --only N >> gpurun_out/ab/gemm.log 2>&1 || exit $?
done
for v in bk32 bk32w4; do
  MDE_LIB=build/var/lib_$v.so timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || exit $?
done

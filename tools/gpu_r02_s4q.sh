#!/bin/bash
# attention: static s_setprio for one half of the waves (variant libraries), kernel timing + B=28 bench
set -o pipefail
o=gpurun_out/s4q; mkdir -p $o
for r in 1 2; do
for v in base prio1 prio2; do
  lib=monocular_depth_estimation_trt_amd/libmde_hip.so; [ $v != base ] && lib=build/var/lib_$v.so
  echo "== $v" >> $o/attn.log
  timeout -k 10 120 python tools/bench_kernels.py --lib $lib --batch 28 --only attention --iters 50 >> $o/attn.log 2>&1 || exit $?
done
done

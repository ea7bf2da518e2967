# GPU-box helper: time tools/bench_kernels.py under the product build and
# the tuning variants build/var/lib_<v>.so given as arguments.
set -e
mkdir -p gpurun_out/ab
for v in base "$@"; do
  lib=monocular_depth_estimation_trt_amd/libmde_hip.so
  [ $v != base ] && lib=build/var/lib_$v.so
  echo "== $v" >> gpurun_out/ab/gemm.log
  timeout -k 10 120 python tools/bench_kernels.py --lib $lib --iters 30 >> gpurun_out/ab/gemm.log 2>&1
done

# GPU-box helper: time the product build and tuning-variant builds (build/var/lib_*.so)
# with tools/bench_kernels.py, then run the GPU tests and the bench.
# Usage (on the box): bash tools/kernel_variants.sh [variant ...]
set -e
mkdir -p gpurun_out
for v in base "$@"; do
  lib=monocular_depth_estimation_trt_amd/libmde_hip.so
  [ $v != base ] && lib=build/var/lib_$v.so
  echo "== $v" >> gpurun_out/kv.log
  timeout -k 10 120 python tools/bench_kernels.py --lib $lib --iters 30 >> gpurun_out/kv.log 2>&1
done
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/kv_tests.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_kv.json 2> gpurun_out/bench_kv.err

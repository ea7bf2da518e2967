set -o pipefail
O=gpurun_out/r6s31
mkdir -p $O
for it in 1 2 3; do
  for L in build/var/att_head.so monocular_depth_estimation_trt_amd/libmde_hip.so; do
    timeout -k 10 120 python tools/bench_kernels.py --lib $L --batch 48 --iters 40 --only attention --attn-cfgs 8m,8m > $O/kern_$(basename $L .so)_$it.log 2>&1 || exit 1
  done
done

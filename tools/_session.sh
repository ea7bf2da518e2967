set -o pipefail
O=gpurun_out/r6s26
mkdir -p $O
for it in 1 2; do
  for L in monocular_depth_estimation_trt_amd/libmde_hip.so build/var/lib_a16_noexp.so build/var/lib_a16_nopv.so build/var/lib_a16_noqk.so build/var/lib_a16_nomax.so build/var/lib_attn_nosync.so; do
    timeout -k 10 120 python tools/bench_kernels.py --lib $L --batch 48 --iters 40 --only attention --attn-cfgs 8m,8m > $O/kern_$(basename $L .so)_$it.log 2>&1 || exit 1
  done
done

set -o pipefail
O=gpurun_out/r6s17
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:upconv" || exit 1
for it in 1; do
  for v in mfma valu; do
    if [ $v = mfma ]; then L=monocular_depth_estimation_trt_amd/libmde_hip.so; else L=build/var/upv_valu.so; fi
    timeout -k 10 120 python tools/bench_kernels.py --batch 48 --iters 20 --lib $L --only head > $O/kern_${v}_$it.log 2>&1 || exit 1
    timeout -k 10 300 python -u tools/bench_lib.py $L --steps 40 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/bench_${v}_$it.json 2> $O/bench_${v}_$it.err || exit 1
  done
done

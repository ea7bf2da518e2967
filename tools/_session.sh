set -o pipefail
O=gpurun_out/r6s18
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:attention or bench_batches or b48_replays or vs_golden_518 or graph" || exit 1
for it in 1 2; do
  for v in sum max; do
    if [ $v = sum ]; then L=monocular_depth_estimation_trt_amd/libmde_hip.so; else L=build/var/att_max.so; fi
    timeout -k 10 120 python tools/bench_kernels.py --batch 48 --iters 40 --lib $L --only attention > $O/kern_${v}_$it.log 2>&1 || exit 1
    timeout -k 10 300 python -u tools/bench_lib.py $L --steps 40 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/bench_${v}_$it.json 2> $O/bench_${v}_$it.err || exit 1
  done
done

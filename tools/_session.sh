set -o pipefail
O=gpurun_out/r6s23
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:attention or bench_batches or b48_replays or vs_golden_518 or graph" || exit 1
for it in 1 2; do
  timeout -k 10 120 python tools/bench_kernels.py --batch 48 --iters 40 --only attention --attn-cfgs 8,8m,8,8m > $O/kern_$it.log 2>&1 || exit 1
  for v in 0 1; do
    MDE_ATTN16=$v timeout -k 10 300 python -u bench.py --steps 40 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/bench_${v}_$it.json 2> $O/bench_${v}_$it.err || exit 1
  done
done

set -o pipefail
O=gpurun_out/r6s24
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:attention or split or b1 or vitl or size_sweep or narrow" || exit 1
for it in 1 2; do
  timeout -k 10 120 python tools/bench_kernels.py --batch 1 --iters 100 --only attention --attn-cfgs 8g4,8g4m,8g4,8g4m > $O/kern_s_$it.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_kernels.py --batch 1 --dim 1024 --heads 16 --iters 100 --only attention --attn-cfgs 8g2,8g2m,8g2,8g2m > $O/kern_l_$it.log 2>&1 || exit 1
  for v in 0 1; do
    MDE_ATTN16=$v timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/bench_${v}_$it.json 2> $O/bench_${v}_$it.err || exit 1
    MDE_ATTN16=$v timeout -k 10 300 python -u bench.py --encoder vitl --global-batch 1 --steps 20 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/benchl_${v}_$it.json 2> $O/benchl_${v}_$it.err || exit 1
  done
done

set -o pipefail
O=gpurun_out/r6s15
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:tile96 or qkv_layout or vs_golden_518" || exit 1
for it in 1 2; do
  for v in 0 1; do
    MDE_TILE96=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 100 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/b1_t${v}_$it.json 2> $O/b1_t${v}_$it.err || exit 1
  done
done

set -o pipefail
O=gpurun_out/r6s13
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:narrow_resid or reference_size_sweep or fc2_splitk or vs_golden_518 or test_linear_residual or panel32" || exit 1
for it in 1 2; do
  for v in 0 1; do
    MDE_NARROW_RESID=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 100 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/b1_n${v}_$it.json 2> $O/b1_n${v}_$it.err || exit 1
  done
done

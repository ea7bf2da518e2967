# GPU-box helper: time the attention kernel under each MDE_ATTN_CFG (B=32 and B=1)
set -e
mkdir -p gpurun_out
for cfg in 16x8 16x4 32x4 16x2; do
  for b in 30 1; do
    echo "== $cfg B=$b" >> gpurun_out/attn.log
    MDE_ATTN_CFG=$cfg timeout -k 10 120 python tools/bench_kernels.py --batch $b --only attention --iters 50 >> gpurun_out/attn.log 2>&1
  done
done

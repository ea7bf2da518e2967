set -o pipefail
O=gpurun_out/r5s4
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:attention" \
  bench:pk1:--no-b1,--no-cpu-baseline env:MDE_ATTN_PACK=0 bench:pk0:--no-b1,--no-cpu-baseline unenv:MDE_ATTN_PACK \
  bench:pk1b:--no-b1,--no-cpu-baseline env:MDE_ATTN_PACK=0 bench:pk0b:--no-b1,--no-cpu-baseline unenv:MDE_ATTN_PACK \
  kern:a6:--batch,48,--iters,50,--only,attention,--attn-cfgs,8+8p+8+8p+8+8p

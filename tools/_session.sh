set -o pipefail
O=gpurun_out/r5s5
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:attention_swp or attention_tuning" \
  kern:a7:--batch,48,--iters,50,--only,attention,--attn-cfgs,8+8w+8+8w+8+8w \
  env:MDE_ATTN_SWP=1 bench:w1:--no-b1,--no-cpu-baseline,--no-pcie unenv:MDE_ATTN_SWP bench:w0:--no-b1,--no-cpu-baseline,--no-pcie \
  env:MDE_ATTN_SWP=1 bench:w1b:--no-b1,--no-cpu-baseline,--no-pcie unenv:MDE_ATTN_SWP bench:w0b:--no-b1,--no-cpu-baseline,--no-pcie \
  env:MDE_CONV_PERSIST=0 bench:cp0:--no-b1,--no-cpu-baseline,--no-pcie unenv:MDE_CONV_PERSIST bench:cp1:--no-b1,--no-cpu-baseline,--no-pcie \
  env:MDE_CONV_PERSIST=0 bench:cp0b:--no-b1,--no-cpu-baseline,--no-pcie unenv:MDE_CONV_PERSIST bench:cp1b:--no-b1,--no-cpu-baseline,--no-pcie

#!/bin/bash
# round-3 session 5: full GPU suite (deep ring on im2col split-K, slice-aware
# XCD order, 8g4 default for ViT-S B=1, 8-wave small-grid 128^2), B=1 A/Bs
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s5 tests smoke \
  bench:vits1:--batch,1,--no-cpu-baseline,--no-b1 \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_GEMM_W8SMALL=0 bench:vitl1now8:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_GEMM_W8SMALL \
  env:MDE_ATTN_CFG=12g3 bench:vitl1g123:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=16g4 bench:vitl1g164:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  bench:vitl1b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  bench:def:--no-cpu-baseline

#!/bin/bash
# round-3 session 3: smoke-order diagnosis, new GPU tests, B=1 ViT-L A/Bs
set -o pipefail
bash tools/diag_smoke.sh || exit 1
bash tools/gpu_tasks.sh gpurun_out/r3s3 "tests:tile_variants or key_groups or dpt_fork" smoke \
  bench:def:--no-cpu-baseline \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_DPT_FORK=0 bench:vitl1nofork:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_DPT_FORK \
  env:MDE_ATTN_CFG=4g2 bench:vitl1g42:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=8g2 bench:vitl1g82:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  env:MDE_GEMM_TILE=128x128w8 bench:vitl1w8:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_GEMM_TILE=big1 bench:vitl1big:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_GEMM_TILE \
  bench:vitl1b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1

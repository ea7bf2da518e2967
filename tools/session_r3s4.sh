#!/bin/bash
# round-3 session 4: full GPU suite with the key-group default and deep 64^2
# rings, ViT-S / ViT-L B=1 A/Bs, ViT-L B=1 rocprof/PMC evidence
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s4 tests smoke \
  bench:def:--no-cpu-baseline \
  bench:vits1:--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_GEMM_DEEP64=0 bench:vits1nodeep:--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_GEMM_DEEP64 \
  env:MDE_ATTN_CFG=8g4 bench:vits1g84:--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=4g2 bench:vits1g42:--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_GEMM_DEEP64=0 bench:vitl1nodeep:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_GEMM_DEEP64 \
  env:MDE_ATTN_CFG=4s2 bench:vitl1s2:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  bench:vitl1b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  profile:vitl1:--encoder,vitl,--batch,1

#!/bin/bash
# round-3 session 4: full GPU suite with the key-group default, ViT-S B=1
# attention A/B, ViT-L B=1 with the new defaults + its rocprof/PMC evidence
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s4 tests smoke \
  bench:def:--no-cpu-baseline \
  bench:vits1:--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=8g4 bench:vits1g84:--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=4g2 bench:vits1g42:--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=8g2 bench:vits1g82:--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  bench:vits1b:--batch,1,--no-cpu-baseline,--no-b1 \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_ATTN_CFG=4s2 bench:vitl1s2:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_ATTN_CFG \
  profile:vitl1:--encoder,vitl,--batch,1

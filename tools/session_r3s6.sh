#!/bin/bash
# round-3 session 6: small-grid split / conv-tile A/Bs at batch 1, default
# bench, upconv restructure (hoisted column work) vs HEAD + ablations at B=48
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s6 "tests:splitk or conv3x3 or engine_vs or fc2_splitk or tile_variants or depth_head or upconv" \
  "kern:new:--batch,48,--only,head" "kern:old:--batch,48,--only,head,--lib,build/var/lib_rev_HEAD.so" \
  "kern:nomfma:--batch,48,--only,head,--lib,build/var/lib_conv_nomfma.so" \
  "kern:nov:--batch,48,--only,head,--lib,build/var/lib_upconv_nov.so" \
  "kern:noh:--batch,48,--only,head,--lib,build/var/lib_upconv_noh.so" "kern:new2:--batch,48,--only,head" \
  bench:vits1:--batch,1,--no-cpu-baseline,--no-b1 bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  env:MDE_CONV_BN64=0 bench:vitl1nb64:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_CONV_BN64 \
  env:MDE_GEMM_DEEP64=0 bench:vitl1nd:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  bench:vits1nd:--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_GEMM_DEEP64 \
  bench:vitl1b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 bench:def:--no-cpu-baseline

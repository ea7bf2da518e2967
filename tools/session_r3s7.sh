#!/bin/bash
# round-3 session 7: tap LayerNorm folded into the DPT projects -- engine GPU
# tests, then new vs HEAD library (MDE_LIB) at B=48 and B=1, same box
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s7 "tests:engine or dropin or depth or lnfold" \
  bench:new:--no-cpu-baseline,--no-b1 env:MDE_LIB=build/var/lib_rev_HEAD.so bench:old:--no-cpu-baseline,--no-b1 \
  bench:oldl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 unenv:MDE_LIB \
  bench:newl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 bench:new2:--no-cpu-baseline,--no-b1

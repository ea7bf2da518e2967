#!/bin/bash
# round-3 evidence session: full GPU suite, smoke, default bench (+CPU
# baseline), its rocprof stats + FETCH/WRITE passes, config 3's unit (ViT-L
# B=1) bench + profile, Depth Pro and VGGT bench lines
set -o pipefail
O=${1:-gpurun_out/r3ev}
bash tools/gpu_tasks.sh $O tests smoke \
  bench:def: \
  profile:def \
  bench:vitl1:--encoder,vitl,--batch,1 \
  profile:vitl1:--encoder,vitl,--batch,1 \
  bench:dp:--model,depth_pro,--no-cpu-baseline \
  bench:vggt:--model,vggt,--no-cpu-baseline

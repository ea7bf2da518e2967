#!/bin/bash
# Round evidence session: full GPU suite, smoke, default bench (+CPU
# baseline), its rocprof kernel stats + FETCH/WRITE passes (traffic JSON) and
# SQ counter passes (PMC table), config 3's unit (ViT-L B=1), the fp32 engine,
# the reference's size sweep, Depth Pro and VGGT bench lines.
#   bash tools/session_evidence.sh OUT
set -o pipefail
O=${1:-gpurun_out/ev}
bash tools/gpu_tasks.sh $O tests smoke \
  bench:def: \
  profile:def \
  pmc:def: \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie \
  bench:fp32:--precision,fp32,--batch,8,--no-cpu-baseline,--no-pcie \
  bench:s392:--size,392x518,--no-cpu-baseline,--no-pcie \
  bench:s672:--size,672x896,--no-cpu-baseline,--no-pcie \
  bench:dp:--model,depth_pro,--no-cpu-baseline,--no-pcie \
  bench:vggt:--model,vggt,--no-cpu-baseline,--no-pcie

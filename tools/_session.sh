set -o pipefail
O=gpurun_out/r5s9
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:l2pf or small_grid_variants or linear_splitk or fc2_splitk" \
  kern:p0:--dim,1024,--heads,16,--batch,1,--only,N3072,--cold env:MDE_L2PF=1 kern:p1:--dim,1024,--heads,16,--batch,1,--only,N3072,--cold unenv:MDE_L2PF \
  bench:l0:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie env:MDE_L2PF=1 bench:l1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie unenv:MDE_L2PF \
  bench:l0b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie env:MDE_L2PF=1 bench:l1b:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie unenv:MDE_L2PF

set -o pipefail
O=gpurun_out/r6ev2b
mkdir -p $O
bash tools/gpu_tasks.sh $O bench:def: \
  bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie \
  bench:fp32:--precision,fp32,--batch,8,--no-cpu-baseline,--no-pcie \
  bench:s392:--size,392x518,--no-cpu-baseline,--no-pcie \
  bench:s672:--size,672x896,--no-cpu-baseline,--no-pcie \
  bench:dp:--model,depth_pro,--no-cpu-baseline,--no-pcie \
  bench:vggt:--model,vggt,--no-cpu-baseline,--no-pcie || exit 1

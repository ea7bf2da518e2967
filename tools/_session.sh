set -o pipefail
O=gpurun_out/r4e5
mkdir -p $O
bash tools/gpu_tasks.sh $O tests smoke bench:def: bench:b1:--batch,1,--no-cpu-baseline bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline

set -o pipefail
O=gpurun_out/r5s1
mkdir -p $O
bash tools/gpu_tasks.sh $O probe:p:4000,20 kpmc:attn48:--batch,48,--only,attention bench:def: bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline

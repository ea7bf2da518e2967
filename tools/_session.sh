set -o pipefail
O=gpurun_out/r6s14
mkdir -p $O
bash tools/gpu_tasks.sh $O tests smoke bench:def: bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie "kern:attn_b1:--batch,1,--iters,50,--only,attention,--attn-cfgs,8g4+4s2+4s3+4s4+8s2+8s3+4g4+8g2" || exit 1

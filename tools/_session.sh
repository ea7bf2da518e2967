set -o pipefail
O=gpurun_out/r5s3
mkdir -p $O
bash tools/gpu_tasks.sh $O "tests:conv3x3_32 or conv_transpose32 or resize32 or fp32_precision or linear32 or attention32 or qkv32" \
  bench:fp32:--precision,fp32,--batch,8,--no-cpu-baseline \
  trace:pcie:--steps,10,--warmup,3 \
  kern:a5:--batch,48,--iters,50,--only,attention,--attn-cfgs,8+4q2+8+4q2+8+4q2 \
  pmc:def:

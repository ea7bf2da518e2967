set -o pipefail
O=gpurun_out/r4s4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -m gpu -v -s --timeout 300 --timeout-method thread -k "fp32" > $O/fp32.log 2>&1 || exit 1
bash tools/gpu_tasks.sh $O bench:f32:--no-cpu-baseline,--precision,fp32,--batch,8,--steps,5 bench:f32l1:--no-cpu-baseline,--precision,fp32,--batch,1,--encoder,vitl,--steps,5,--no-b1

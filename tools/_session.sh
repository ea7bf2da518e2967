set -o pipefail
O=gpurun_out/r4s5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "mlp_fused or bench_batches" > $O/mlp.log 2>&1 || exit 1
bash tools/gpu_tasks.sh $O bench:fused:--no-cpu-baseline,--no-b1 env:MDE_MLPFUSE=0 bench:unfused:--no-cpu-baseline,--no-b1 unenv:MDE_MLPFUSE env:MDE_LIB=build/var/lib_conv_tall.so tests:conv3x3 bench:tall:--no-cpu-baseline,--no-b1 unenv:MDE_LIB bench:fused2:--no-cpu-baseline,--no-b1

#!/bin/bash
# row-block GEMM: op parity, engine parity, bench, kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "ln_ or residual_f16" > gpurun_out/rb_ops.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
MDE_RB_PROJ=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-b1 > gpurun_out/bench_noproj.json 2> gpurun_out/bench_noproj.err || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-b1 --no-cpu-baseline --profile-iters 1 > gpurun_out/stats.log 2>&1 || exit $?

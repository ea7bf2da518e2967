#!/bin/bash
# conv ReLU-once + no-NaN build, V^T staged epilogue: tests, bench, stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "qkv or conv or depth_head" > gpurun_out/ops.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-b1 --no-cpu-baseline --profile-iters 1 > gpurun_out/stats.log 2>&1 || exit $?

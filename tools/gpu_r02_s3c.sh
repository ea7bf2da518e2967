#!/bin/bash
# conv up-blend rewrite (product) + attention f16 row-sum variant (build/var)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
export MDE_LIB=build/var/lib_attnf16.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread -k "attention or engine" -s > gpurun_out/attnf16_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-b1 > gpurun_out/bench_attnf16.json 2> gpurun_out/bench_attnf16.err || exit $?
unset MDE_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread -s > gpurun_out/engine_base.log 2>&1 || exit $?

#!/bin/bash
# batched bias / LN-partial loads (one round trip): parity, then same-box A/B vs v3 lib
set -o pipefail
o=gpurun_out/s3l; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit $?
MDE_LIB=build/var/lib_v3.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_v3.json 2> $o/bench_v3.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench2.json 2> $o/bench2.err || exit $?

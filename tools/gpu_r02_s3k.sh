#!/bin/bash
# LN fold v3 (rows split over waves, LDS exchange): parity, then same-box A/B vs no-fold and no-loads variant
set -o pipefail
o=gpurun_out/foldexp2; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -s -k "lnfold or residual_f16 or engine or patch_embed or qkv" > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit $?
MDE_LIB=build/var/lib_foldexp.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-b1 > $o/bench_exp.json 2> $o/bench_exp.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_nofold.json 2> $o/bench_nofold.err || exit $?

#!/bin/bash
# LayerNorm folded across the GEMM boundaries: op parity, engine parity, A/B bench (B=28 and B=1)
set -o pipefail
mkdir -p gpurun_out/fold
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "lnfold or residual_f16 or qkv or patch_embed" > gpurun_out/fold/ops.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -s > gpurun_out/fold/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/fold/bench.json 2> gpurun_out/fold/bench.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/fold/bench_nofold.json 2> gpurun_out/fold/bench_nofold.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > gpurun_out/fold/vitl_b1.json 2> gpurun_out/fold/vitl_b1.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > gpurun_out/fold/vitl_b1_nofold.json 2> gpurun_out/fold/vitl_b1_nofold.err || exit $?

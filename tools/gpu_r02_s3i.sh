#!/bin/bash
# LN fold v2 (one-round-trip partial loads): A/B benches, then the fold parity tests
set -o pipefail
mkdir -p gpurun_out/fold7
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/fold7/bench.json 2> gpurun_out/fold7/bench.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/fold7/bench_nofold.json 2> gpurun_out/fold7/bench_nofold.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > gpurun_out/fold7/vitl_b1.json 2> gpurun_out/fold7/vitl_b1.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > gpurun_out/fold7/vitl_b1_nofold.json 2> gpurun_out/fold7/vitl_b1_nofold.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -k "lnfold or residual_f16 or engine or patch_embed" > gpurun_out/fold7/tests.log 2>&1 || exit $?

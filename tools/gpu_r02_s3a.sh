#!/bin/bash
# round-2 session-3 baseline: GPU tests, default bench, SQ/TCC counter passes at B=28, b1 layers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
bash tools/pmc_profile.sh gpurun_out/pmc_b28 -- python3 bench.py --steps 3 --warmup 1 --no-b1 --no-cpu-baseline --profile-iters 1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_b28 > gpurun_out/pmc_b28_summary.txt || exit $?
bash tools/b1_layers.sh

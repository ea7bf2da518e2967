#!/bin/bash
# batch-1 kernel traces (graph replay) for ViT-S and ViT-L
set -o pipefail
mkdir -p gpurun_out/b1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b1/vits -o run --output-format csv -- python3 bench.py --batch 1 --steps 30 --warmup 5 --no-b1 --no-cpu-baseline --profile-iters 1 > gpurun_out/b1/vits.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b1/vitl -o run --output-format csv -- python3 bench.py --encoder vitl --batch 1 --steps 30 --warmup 5 --no-b1 --no-cpu-baseline --profile-iters 1 > gpurun_out/b1/vitl.log 2>&1 || exit $?

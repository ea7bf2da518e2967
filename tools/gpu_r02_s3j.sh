#!/bin/bash
# LN fold for D <= 1024: parity (ops + engines), A/B at ViT-S B=28, ViT-L B=1 and B=8
set -o pipefail
o=gpurun_out/fold9; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -x -q --timeout 200 --timeout-method thread -s -k "lnfold or residual_f16 or engine or patch_embed" > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench.json 2> $o/bench.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_nofold.json 2> $o/bench_nofold.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > $o/vitl_b1.json 2> $o/vitl_b1.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 > $o/vitl_b1_nofold.json 2> $o/vitl_b1_nofold.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 8 --no-b1 --no-cpu-baseline --steps 10 > $o/vitl_b8.json 2> $o/vitl_b8.err || exit $?
MDE_LNFOLD=0 timeout -k 10 300 python -u bench.py --encoder vitl --batch 8 --no-b1 --no-cpu-baseline --steps 10 > $o/vitl_b8_nofold.json 2> $o/vitl_b8_nofold.err || exit $?

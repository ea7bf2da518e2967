#!/bin/bash
# small-batch breakdowns: ViT-L B=1 (config 3's unit) and ViT-S B=1, per-layer classes + rocprof kernel stats
set -o pipefail
o=gpurun_out/s4c; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline --layers-json $o/vitl_b1_layers.json > $o/vitl_b1.json 2> $o/vitl_b1.err || exit $?
timeout -k 10 300 python -u bench.py --batch 1 --steps 30 --no-b1 --no-cpu-baseline --layers-json $o/vits_b1_layers.json > $o/vits_b1.json 2> $o/vits_b1.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_vitl_b1 -o run --output-format csv -- python3 bench.py --encoder vitl --batch 1 --steps 10 --warmup 2 --no-b1 --no-cpu-baseline --profile-iters 1 > $o/prof_vitl_b1.log 2>&1 || exit $?

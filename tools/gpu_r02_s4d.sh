#!/bin/bash
# E_STORE split-K: op parity, engine parity, small-batch and default benches with MDE_SPLITK on/off
set -o pipefail
o=gpurun_out/s4d; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "splitk or conv3x3 or linear" -x -q --timeout 120 --timeout-method thread > $o/ops.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $o/engine.log 2>&1 || exit $?
for enc in vitl vits; do
  timeout -k 10 300 python -u bench.py --encoder $enc --batch 1 --steps 30 --no-b1 --no-cpu-baseline --layers-json $o/${enc}_b1_layers.json > $o/${enc}_b1.json 2> $o/${enc}_b1.err || exit $?
  MDE_SPLITK=0 timeout -k 10 300 python -u bench.py --encoder $enc --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/${enc}_b1_nosplit.json 2> $o/${enc}_b1_nosplit.err || exit $?
done
timeout -k 10 300 python -u bench.py --encoder vitl --batch 8 --steps 20 --no-b1 --no-cpu-baseline > $o/vitl_b8.json 2> $o/vitl_b8.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/vits_b28.json 2> $o/vits_b28.err || exit $?

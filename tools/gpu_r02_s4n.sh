#!/bin/bash
# fused split-K fixup (last slice workgroup per tile runs the reduce + epilogue): parity and batch-1 benches
set -o pipefail
o=gpurun_out/s4n; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for enc in vitl vits; do
  timeout -k 10 300 python -u bench.py --encoder $enc --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/${enc}_b1.json 2> $o/${enc}_b1.err || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/vits_b28.json 2> $o/vits_b28.err || exit $?

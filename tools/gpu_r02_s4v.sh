#!/bin/bash
# attention split policy (>= 7 tiles per split, <= ~400 workgroups): parity + batch-1/2 benches
set -o pipefail
o=gpurun_out/s4v; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_engine.py -k "attention or 518 or consistency or splitk" -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for a in "--batch 1" "--batch 2" "--encoder vitl --batch 1"; do
  tag=$(echo $a | tr -d ' -')
  timeout -k 10 300 python -u bench.py $a --steps 40 --no-b1 --no-cpu-baseline > $o/$tag.json 2> $o/$tag.err || exit $?
  python -c "import json;d=json.load(open('$o/$tag.json'));print('$tag',d['value'],d['ms_per_step'])" >> $o/summary.txt
done

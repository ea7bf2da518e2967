#!/bin/bash
# same-box A/B of the default batch: 28 vs 40 vs 48, alternating, three passes
set -o pipefail
o=gpurun_out/s4ad; mkdir -p $o
for r in 1 2 3; do
for b in 28 40 48; do
  timeout -k 10 300 python -u bench.py --batch $b --no-b1 --no-cpu-baseline > $o/b${b}_$r.json 2> $o/b${b}_$r.err || exit $?
  python -c "import json;d=json.load(open('$o/b${b}_$r.json'));print($b,$r,d['value'],d['ms_per_step'])" >> $o/summary.txt
done
done

#!/bin/bash
# fine batch sweep around the default (fc2 at B=48 = 1542 128^2 tiles = 3.01 rounds of 512)
set -o pipefail
o=gpurun_out/s4af; mkdir -p $o
for r in 1 2; do
for b in 44 46 47 48; do
  timeout -k 10 300 python -u bench.py --batch $b --no-b1 --no-cpu-baseline > $o/b${b}_$r.json 2> $o/b${b}_$r.err || exit $?
  python -c "import json;d=json.load(open('$o/b${b}_$r.json'));print($b,$r,d['value'],d['ms_per_step'])" >> $o/summary.txt
done
done

#!/bin/bash
# E_STORE split-K: minimum K-steps before a small grid splits (MDE_SPLIT_NKMIN 8 / 12 / 16), batch 1
set -o pipefail
o=gpurun_out/s4w; mkdir -p $o
for r in 1 2; do
for v in 8 12 16; do
  for a in "--batch 1" "--encoder vitl --batch 1"; do
    tag=$(echo $a | tr -d ' -')_$v
    MDE_SPLIT_NKMIN=$v timeout -k 10 300 python -u bench.py $a --steps 40 --no-b1 --no-cpu-baseline > $o/$tag.json 2> $o/$tag.err || exit $?
    python -c "import json;d=json.load(open('$o/$tag.json'));print('$tag',d['value'],d['ms_per_step'])" >> $o/summary.txt
    grep -E "\] (rcu.conv|layer_rn) " $o/$tag.err >> $o/summary.txt
  done
done
done

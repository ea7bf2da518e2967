#!/bin/bash
# batch-1 ViT-S attention split count (MDE_ATTN_CFG 4s<k>) vs the default (4s4)
set -o pipefail
o=gpurun_out/s4u; mkdir -p $o
for c in def 4s2 4s3 4s6 def; do
  if [ $c = def ]; then unset MDE_ATTN_CFG; else export MDE_ATTN_CFG=$c; fi
  timeout -k 10 300 python -u bench.py --batch 1 --steps 40 --no-b1 --no-cpu-baseline > $o/vits_$c.json 2> $o/vits_$c.err || exit $?
  grep -E "\] attn " $o/vits_$c.err >> $o/summary.txt
  python -c "import json;d=json.load(open('$o/vits_$c.json'));print('$c',d['value'],d['ms_per_step'])" >> $o/summary.txt
done

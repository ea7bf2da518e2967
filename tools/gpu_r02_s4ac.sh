#!/bin/bash
# larger-batch sweep of the default ViT-S bench (48..96), then rocprof stats + PMC traffic at the best batch
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/s4ac; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "conv3x3" -x -q --timeout 120 --timeout-method thread > $o/convtests.log 2>&1 || exit $?
for b in 48 56 64 72 84 96; do
  timeout -k 10 300 python -u bench.py --batch $b --no-b1 --no-cpu-baseline > $o/b${b}.json 2> $o/b${b}.err || exit $?
  python -c "import json;d=json.load(open('$o/b${b}.json'));print($b,d['value'],d['ms_per_step'])" >> $o/summary.txt
done
best=$(sort -k2 -n -r $o/summary.txt | head -n 1 | cut -d' ' -f1)
echo "best $best" >> $o/summary.txt
bash tools/profile_round.sh $o/prof --batch $best || exit $?

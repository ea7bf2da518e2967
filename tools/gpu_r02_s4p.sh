#!/bin/bash
# batch-1 ViT-L: proj on the split-K path (MDE_SPLITK_PROJ), attention split / wave configs
set -o pipefail
o=gpurun_out/s4p; mkdir -p $o
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/base.json 2> $o/base.err || exit $?
MDE_SPLITK_PROJ=1 timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/proj.json 2> $o/proj.err || exit $?
for c in 4s4 8s4 8s8 4s1; do
  MDE_ATTN_CFG=$c timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/attn_$c.json 2> $o/attn_$c.err || exit $?
done
for c in 4s8 8s8; do
  MDE_ATTN_CFG=$c timeout -k 10 300 python -u bench.py --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vits_attn_$c.json 2> $o/vits_attn_$c.err || exit $?
done
timeout -k 10 300 python -u bench.py --batch 1 --steps 30 --no-b1 --no-cpu-baseline > $o/vits_base.json 2> $o/vits_base.err || exit $?

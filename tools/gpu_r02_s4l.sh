#!/bin/bash
# E_STORE split-K in the VGGT and Depth Pro forwards: parity, then bench with MDE_SPLITK on/off (b1 legs included)
set -o pipefail
o=gpurun_out/s4l; mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_vggt.py tests/test_gpu_depth_pro.py -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
for m in vggt depth_pro; do
  timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > $o/${m}.json 2> $o/${m}.err || exit $?
  MDE_SPLITK=0 timeout -k 10 400 python -u bench.py --model $m --no-cpu-baseline > $o/${m}_nosplit.json 2> $o/${m}_nosplit.err || exit $?
done

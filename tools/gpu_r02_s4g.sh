#!/bin/bash
# in-graph cost of the GEMM epilogues at B=28: main-loop-only and no-GELU variant libraries (timing only)
set -o pipefail
o=gpurun_out/s4g; mkdir -p $o
timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/base.json 2> $o/base.err || exit $?
for v in noepi nogelu; do
  MDE_LIB=build/var/lib_$v.so timeout -k 10 300 python -u bench.py --no-b1 --no-cpu-baseline > $o/$v.json 2> $o/$v.err || exit $?
done

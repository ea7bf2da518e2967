#!/bin/bash
# default bench (B=48) and its rocprof kernel stats + PMC traffic from the same box
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/s4ag; mkdir -p $o
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
bash tools/profile_round.sh $o/prof --batch 48 || exit $?

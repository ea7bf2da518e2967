#!/bin/bash
# A/B session: GPU tests for the change, then the default bench with and
# without it (same box).  usage: bash tools/session_ab.sh OUT 'TEST_EXPR' ENVVAR=OFFVAL [bench args]
set -o pipefail
O=$1; K=$2; OFF=$3; shift 3
A=$(IFS=,; echo "$*")
bash tools/gpu_tasks.sh $O "tests:$K" \
  bench:on:--no-cpu-baseline${A:+,$A} env:$OFF bench:off:--no-cpu-baseline${A:+,$A} unenv:${OFF%%=*} \
  bench:on2:--no-cpu-baseline${A:+,$A}

#!/bin/bash
# refresh the round's evidence for the current code: full GPU suite, smoke, default bench, rocprof stats + PMC traffic
set -o pipefail
o=gpurun_out/s4i; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
bash tools/profile_round.sh $o/prof || exit $?

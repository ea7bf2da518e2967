#!/bin/bash
# final evidence for the session's code: full GPU suite, smoke, default bench, rocprof stats + PMC traffic, ViT-L B=1 line
set -o pipefail
o=gpurun_out/s4x; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --steps 30 > $o/vitl_b1.json 2> $o/vitl_b1.err || exit $?
bash tools/profile_round.sh $o/prof || exit $?
timeout -k 10 300 python -u bench.py --batch 1 --steps 40 --no-cpu-baseline > $o/vits_b1.json 2> $o/vits_b1.err || exit $?

#!/bin/bash
# final check of the round's default: full GPU suite, smoke, default bench (B=48) with b1 and CPU legs, B=28 reference
set -o pipefail
o=gpurun_out/s4ae; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
timeout -k 10 300 python -u bench.py --batch 28 --no-b1 --no-cpu-baseline > $o/bench_b28.json 2> $o/bench_b28.err || exit $?

#!/bin/bash
# GPU-box helper: the round's committed profiles for a bench workload
# (default: DA-V2 ViT-S 518, B=30):
#   1. rocprofv3 --kernel-trace --stats            -> <out>/stats
#   2. one --pmc pass each for FETCH_SIZE, WRITE_SIZE (kernel-trace only,
#      MI355X_MICROARCH.md: counters in their own runs; TCC can't hold both)
#   3. tools/pmc_traffic.py -> <out>/traffic.json (HBM bytes per launch,
#      FETCH_SIZE x2 on gfx950 for 16-B/lane streaming reads), per kernel and
#      per engine layer of the last forward (the bench's --layers-json order)
# usage: bash tools/profile_round.sh OUTDIR [bench.py args...]
set -o pipefail
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
args=(--steps 5 --warmup 2 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 1 --layers-json "$out/layers.json" "$@")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/stats" -o run --output-format csv -- \
  python3 bench.py "${args[@]}" > "$out/stats.log" 2>&1 || exit $?
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$out/pmc$i" -o pmc --output-format csv -- \
    python3 bench.py "${args[@]}" > "$out/pmc$i.log" 2>&1 || exit $?
  i=$((i+1))
done
python3 tools/pmc_traffic.py "$out" "$out/layers.json" > "$out/traffic.json"

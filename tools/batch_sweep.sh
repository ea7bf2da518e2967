#!/bin/bash
# SURVEY.md 8(d) throughput sweep on one box:
#   ViT-S 518^2 at B in {1,2,4,8,16,32,48,64}, ViT-L 518^2 at B in {1,2,4,8}
# one bench.py line per point (HBM-resident inputs, hipGraph replay), then
# tools/batch_sweep_summary.py folds them into OUT/sweep.json.
#   bash tools/batch_sweep.sh OUT [steps]
set -o pipefail
O=${1:-gpurun_out/sweep}
K=${2:-20}
mkdir -p "$O"
run() {  # tag, args...
  local tag=$1; shift
  echo "[sweep $(date +%T)] $tag $*"
  timeout -k 10 300 python -u bench.py --steps "$K" --warmup 5 --no-b1 --no-cpu-baseline --no-pcie \
    --profile-iters 1 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { echo "[sweep] $tag rc=$?"; tail -5 "$O/$tag.err"; exit 1; }
}
for b in 1 2 4 8 16 32 48 64; do run "vits_b$b" --encoder vits --batch "$b"; done
for b in 1 2 4 8; do run "vitl_b$b" --encoder vitl --batch "$b"; done
python tools/batch_sweep_summary.py "$O" > "$O/sweep.json"

#!/bin/bash
# One parameterised GPU-box session (replaces round 2's one-off tools/gpu_r02_s*.sh).
#
#   bash tools/gpu_tasks.sh OUT task [task ...]
#
# Tasks (run in order, each under its own time limit; the first failure ends
# the session -- no retries, nothing more on the GPU after a fault):
#   tests[:EXPR]          pytest -m gpu (optionally -k EXPR)          -> OUT/tests.log
#   smoke                 __graft_entry__ smoke()                     -> OUT/smoke.log
#   peak                  tools/mfma_peak.hip (f16 MFMA peak)         -> OUT/mfma_peak.json
#   probe[:ITERS,LAUNCHES] tools/dma_war_probe.hip (LDS-DMA address WAR) -> OUT/dma_war_probe.json
#   bench:TAG:ARGS        python bench.py ARGS (ARGS comma-separated) -> OUT/bench_TAG.json/.err
#   benchlib:TAG:LIB,ARGS bench.py ARGS against variant library LIB -> OUT/bench_TAG.json/.err
#   profile:TAG:ARGS      tools/profile_round.sh (stats + FETCH/WRITE passes) -> OUT/prof_TAG/
#   pmc:TAG:ARGS          tools/pmc_profile.sh on bench.py ARGS (SQ/TCC passes) -> OUT/pmc_TAG/
#   kpmc:TAG:ARGS         tools/pmc_profile.sh on tools/bench_kernels.py ARGS    -> OUT/kpmc_TAG/
#   trace:TAG:ARGS        rocprofv3 kernel + memory-copy trace of bench.py ARGS -> OUT/trace_TAG/
#   kern:TAG:ARGS         tools/bench_kernels.py ARGS                 -> OUT/kern_TAG.log
#   env:VAR=VAL           export VAR=VAL for the tasks that follow (e.g. env:MDE_ATTN_CFG=8)
#   unenv:VAR             unset VAR
set -o pipefail
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
log() { echo "[gpu_tasks $(date +%T)] $*" | tee -a "$O/session.log"; }
for t in "$@"; do
  IFS=: read -r name tag rest <<< "$t"
  args=()
  if [ -n "$rest" ]; then IFS=, read -r -a args <<< "$rest"; fi
  log "start $t"
  case $name in
    tests)
      k=(); [ -n "$tag" ] && k=(-k "$tag")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 120 --timeout-method thread "${k[@]}" \
        > "$O/tests.log" 2>&1 || { log "tests rc=$?"; tail -30 "$O/tests.log"; exit 1; } ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > "$O/smoke.log" 2>&1 \
        || { log "smoke rc=$?"; exit 1; } ;;
    peak)
      [ -x build/mfma_peak ] || hipcc -O3 --offload-arch=gfx950 -o build/mfma_peak tools/mfma_peak.hip || exit 1
      timeout -k 10 120 ./build/mfma_peak > "$O/mfma_peak.json" 2> "$O/mfma_peak.err" || { log "peak rc=$?"; exit 1; } ;;
    probe)
      [ -x build/dma_war_probe ] || hipcc -O3 --offload-arch=gfx950 -o build/dma_war_probe tools/dma_war_probe.hip || exit 1
      timeout -k 10 180 ./build/dma_war_probe "${args[@]}" > "$O/dma_war_probe.json" 2> "$O/dma_war_probe.err" \
        || { log "probe rc=$?"; exit 1; } ;;
    bench)
      timeout -k 10 600 python -u bench.py "${args[@]}" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" \
        || { log "bench rc=$?"; tail -20 "$O/bench_$tag.err"; exit 1; } ;;
    benchlib)  # benchlib:TAG:LIB,ARGS -- bench.py against a variant library
      timeout -k 10 600 python -u tools/bench_lib.py "${args[@]}" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" \
        || { log "benchlib rc=$?"; tail -20 "$O/bench_$tag.err"; exit 1; } ;;
    profile)
      bash tools/profile_round.sh "$O/prof_$tag" "${args[@]}" || { log "profile rc=$?"; exit 1; } ;;
    pmc)
      bash tools/pmc_profile.sh "$O/pmc_$tag" -- python3 bench.py --steps 3 --warmup 1 --no-b1 --no-cpu-baseline \
        --no-pcie --profile-iters 1 "${args[@]}" || { log "pmc rc=$?"; exit 1; } ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/trace_$tag" -o tr -- \
        python3 bench.py --no-b1 --no-cpu-baseline --profile-iters 1 "${args[@]}" > "$O/trace_$tag.log" 2>&1 \
        || { log "trace rc=$?"; tail -20 "$O/trace_$tag.log"; exit 1; } ;;
    kpmc)
      bash tools/pmc_profile.sh "$O/kpmc_$tag" -- python3 tools/bench_kernels.py --iters 3 "${args[@]}" \
        || { log "kpmc rc=$?"; exit 1; } ;;
    kern)
      timeout -k 10 300 python -u tools/bench_kernels.py "${args[@]}" > "$O/kern_$tag.log" 2>&1 \
        || { log "kern rc=$?"; tail -20 "$O/kern_$tag.log"; exit 1; } ;;
    env) export "$tag"; log "export $tag" ;;
    unenv) unset "$tag" ;;
    *) log "unknown task $t"; exit 2 ;;
  esac
  log "done $t"
done
log "session complete"

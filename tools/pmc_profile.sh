#!/bin/bash
# Collect PMC counter passes for a command (one rocprofv3 call per pass, as
# MI355X_MICROARCH.md prescribes: counters in their own runs, kernel-trace only).
# usage: tools/pmc_profile.sh OUTDIR -- cmd args...
set -o pipefail
out=$1; shift; shift
export TMPDIR=/tmp
mkdir -p "$out"
passes=(
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES"
 "SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $p -d "$out/p$i" -o pmc --output-format csv -- "$@" > "$out/p$i.log" 2>&1 || exit $?
  i=$((i+1))
done

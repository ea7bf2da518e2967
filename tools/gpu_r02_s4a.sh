#!/bin/bash
# session-4 baseline on a fresh box: GPU tests, default bench, attention SQ counters
set -o pipefail
o=gpurun_out/s4a; mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $o/bench.json 2> $o/bench.err || exit $?
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_SALU,SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU_TRANS_F32,SQ_ACTIVE_INST_FLAT,SQ_INST_CYCLES_VMEM,SQ_WAIT_INST_ANY,GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${set//,/ } -d $o/attn_pmc$i -o pmc --output-format csv -- \
    python3 tools/bench_kernels.py --batch 28 --only attention --iters 3 > $o/attn_pmc$i.log 2>&1
  echo "pass $i rc=$?"
  i=$((i+1))
done
exit 0

# GPU-box helper: SQ counters of the attention kernel (microbenchmark), one pass per counter set
export TMPDIR=/tmp
mkdir -p gpurun_out
cfg=${CFG:-8x2}; b=${B:-28}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_SALU,SQ_ACTIVE_INST_MISC"; do
  MDE_ATTN_CFG=$cfg timeout -s KILL 90 rocprofv3 --kernel-trace --pmc ${set//,/ } -d gpurun_out/attn_pmc$i -o pmc --output-format csv -- \
    python3 tools/bench_kernels.py --batch $b --only attention --iters 3 > gpurun_out/attn_pmc$i.log 2>&1
  echo "pass $i rc=$?"
  i=$((i+1))
done

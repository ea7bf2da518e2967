# GPU-box helper: attention parity, then the kernel timed per MDE_ATTN_CFG (<waves>[s<split>]) and batch
mkdir -p gpurun_out
for c in ${CFGS:-8}; do MDE_ATTN_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention" -v --timeout 120 --timeout-method thread >> gpurun_out/attn_tests.log 2>&1 || exit $?; done
rc=$?; echo "attn tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in ${CFGS:-8 4}; do
  for b in ${BATCHES:-30 28 1}; do
    echo "== cfg $cfg B=$b" >> gpurun_out/attn.log
    MDE_ATTN_CFG=$cfg timeout -k 10 120 python tools/bench_kernels.py --batch $b --only attention --iters 50 >> gpurun_out/attn.log 2>&1 || exit $?
  done
done

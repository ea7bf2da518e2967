# GPU-box: GPU parity tests (metrics printed: -s), then -- only if nothing
# crashed or timed out -- the default bench and a B=28 bench line
mkdir -p gpurun_out
tag=${TAG:-a}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r02_bench_$tag.json 2> gpurun_out/r02_bench_$tag.err || exit $?
echo "bench rc=$?"
if [ -n "$EXTRA_BENCH" ]; then
  timeout -k 10 300 python -u bench.py $EXTRA_BENCH --no-cpu-baseline > gpurun_out/r02_bench_${tag}_x.json 2> gpurun_out/r02_bench_${tag}_x.err || exit $?
fi

set -o pipefail
O=gpurun_out/r4s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_vggt.py tests/test_gpu_engine.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "vggt_1b_full or bench_batches or lnfold_matches or fc2_splitk" > $O/metrics.log 2>&1 || exit 1
bash tools/gpu_tasks.sh $O "tests:conv" bench:new:--no-cpu-baseline,--no-b1 env:MDE_LIB=build/var/lib_rev_HEAD.so bench:old:--no-cpu-baseline,--no-b1 unenv:MDE_LIB bench:new2:--no-cpu-baseline,--no-b1 \
  bench:l1:--no-cpu-baseline,--no-b1,--encoder,vitl,--batch,1,--steps,50 env:MDE_LIB=build/var/lib_gemm_wide_small.so bench:l1wide:--no-cpu-baseline,--no-b1,--encoder,vitl,--batch,1,--steps,50 unenv:MDE_LIB bench:l1b:--no-cpu-baseline,--no-b1,--encoder,vitl,--batch,1,--steps,50

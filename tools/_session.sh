set -o pipefail
O=gpurun_out/r6s7
mkdir -p $O
P=monocular_depth_estimation_trt_amd/libmde_hip.so
for it in 1 2; do
  for v in new attn_prio; do
    if [ $v = new ]; then L=$P; else L=build/var/lib_$v.so; fi
    timeout -k 10 120 python tools/bench_kernels.py --batch 48 --iters 40 --lib $L --only attention > $O/kern_${v}_$it.log 2>&1 || exit 1
    timeout -k 10 300 python -u tools/bench_lib.py $L --steps 40 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 3 > $O/bench_${v}_$it.json 2> $O/bench_${v}_$it.err || exit 1
  done
  for b in 44 46 47 48 50 52; do
    timeout -k 10 300 python -u bench.py --batch $b --steps 40 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 1 > $O/b${b}_$it.json 2> $O/b${b}_$it.err || exit 1
  done
done

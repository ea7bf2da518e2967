set -o pipefail
O=gpurun_out/r6s29
mkdir -p $O
for it in 1 2; do
  for L in monocular_depth_estimation_trt_amd/libmde_hip.so build/var/lib_uc_nov.so build/var/lib_uc_noh.so build/var/lib_uc_nomfma.so; do
    n=$(basename $L .so)
    timeout -k 10 300 python -u tools/bench_lib.py $L --steps 10 --no-b1 --no-cpu-baseline --no-pcie --profile-iters 5 --layers-json $O/layers_${n}_$it.json > $O/bench_${n}_$it.json 2> $O/bench_${n}_$it.err || exit 1
  done
done

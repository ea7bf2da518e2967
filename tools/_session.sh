set -o pipefail
O=gpurun_out/r4s20
mkdir -p $O
timeout -k 10 300 python -u tools/_det.py > $O/det.log 2>&1 || exit 1
timeout -k 10 120 ./build/mlp_probe > $O/probe.log 2>&1 || exit 1
bash tools/gpu_tasks.sh $O bench:fused:--no-cpu-baseline,--no-b1

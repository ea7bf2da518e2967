set -o pipefail
O=gpurun_out/r5s10
mkdir -p $O
A=--no-b1,--no-cpu-baseline,--no-pcie
bash tools/gpu_tasks.sh $O tests smoke bench:b32:--batch,32,$A bench:b40:--batch,40,$A bench:b48:--batch,48,$A bench:b56:--batch,56,$A \
  bench:b64:--batch,64,$A bench:b72:--batch,72,$A bench:b96:--batch,96,$A bench:b48b:--batch,48,$A bench:b64b:--batch,64,$A

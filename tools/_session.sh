set -o pipefail
O=gpurun_out/r5x17
mkdir -p $O
A=--no-b1,--no-cpu-baseline,--no-pcie
bash tools/gpu_tasks.sh $O env:MDE_PANEL=1 bench:pon:$A unenv:MDE_PANEL bench:poff:$A env:MDE_PANEL=1 bench:pon2:$A \
  "tests:engine_518_bench or replays or graph or lnfold or golden_518"

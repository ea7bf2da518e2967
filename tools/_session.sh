set -o pipefail
O=gpurun_out/r5x20
mkdir -p $O
A=--no-b1,--no-cpu-baseline,--no-pcie
bash tools/gpu_tasks.sh $O bench:pon:$A env:MDE_PANEL=0 bench:poff:$A unenv:MDE_PANEL bench:pon2:$A "tests:engine_518_bench or replays or graph or lnfold or golden_518 or panel"

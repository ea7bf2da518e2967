set -o pipefail
O=gpurun_out/r5x24
mkdir -p $O
K=--batch,48,--iters,20,--only,K384
F=--batch,48,--iters,20,--only,fc2
A=--no-b1,--no-cpu-baseline,--no-pcie
bash tools/gpu_tasks.sh $O "tests:panel or test_linear or qkv_layout" kern:pon:$K env:MDE_PANEL=0 kern:poff:$K bench:poff:$A unenv:MDE_PANEL \
  bench:pon:$A benchlib:fw4:build/var/px_fw4.so,$A kern:fbase:$F kern:fw4:$F,--lib,build/var/px_fw4.so \
  "tests:engine_518_bench or replays or graph or lnfold or golden_518"

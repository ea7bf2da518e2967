set -o pipefail
O=gpurun_out/r5x9
mkdir -p $O
K=--batch,48,--iters,20,--only,K384
bash tools/gpu_tasks.sh $O kern:pon:$K env:MDE_PANEL=0 kern:poff:$K unenv:MDE_PANEL "tests:panel or qkv_layout or test_linear"

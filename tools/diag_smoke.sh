mkdir -p gpurun_out/diag
timeout -k 5 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/diag/a_smoke_only.log 2>&1; echo "a rc=$?"
timeout -k 5 120 python -u -c "import torch; torch.cuda.init(); import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/diag/b_torch_first.log 2>&1; echo "b rc=$?"
timeout -k 5 120 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/diag/c_build_smoke.log 2>&1; echo "c rc=$?"
env | grep -i -E "hip|rocr|hsa|cuda|gpu" > gpurun_out/diag/env.txt

# The round-5 closing evidence session (gpurun_out/r5e7 + r5e8): GPU suite,
# smoke, default bench + its rocprof stats and HBM traffic passes (without the
# PCIe leg), ViT-L batch-1 bench, ViT-S batch-1 profile.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/_session.sh'
set -o pipefail
O=gpurun_out/r5e9
mkdir -p $O
bash tools/gpu_tasks.sh $O tests smoke bench:def: profile:def bench:vitl1:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-pcie profile:vits1:--batch,1

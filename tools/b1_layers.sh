mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --batch 1 --no-b1 --no-cpu-baseline --steps 50 --layers-json gpurun_out/b1_vits_layers.json > gpurun_out/b1_vits.json 2> gpurun_out/b1_vits.err || exit $?
timeout -k 10 300 python -u bench.py --encoder vitl --batch 1 --no-b1 --no-cpu-baseline --steps 30 --layers-json gpurun_out/b1_vitl_layers.json > gpurun_out/b1_vitl.json 2> gpurun_out/b1_vitl.err || exit $?

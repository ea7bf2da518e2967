#!/bin/bash
# round-3 session 9: 3-deep 64^2 ring for 512-768-tile grids, 32-wide conv
# tiles for tiny 64-channel grids -- GPU tests, then new vs HEAD library
set -o pipefail
bash tools/gpu_tasks.sh gpurun_out/r3s9 "tests:conv3x3 or engine or tile_variants or splitk or linear" \
  bench:s1new:--batch,1,--no-cpu-baseline,--no-b1 env:MDE_LIB=build/var/lib_rev_HEAD.so \
  bench:s1old:--batch,1,--no-cpu-baseline,--no-b1 bench:l1old:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 \
  bench:defold:--no-cpu-baseline,--no-b1 unenv:MDE_LIB \
  bench:l1new:--encoder,vitl,--batch,1,--no-cpu-baseline,--no-b1 bench:defnew:--no-cpu-baseline,--no-b1 \
  bench:s1new2:--batch,1,--no-cpu-baseline,--no-b1

set -o pipefail
O=gpurun_out/r5s8
mkdir -p $O
run() { echo "== $*" >> $O/ring.log; timeout -k 5 60 "$@" >> $O/ring.log 2>&1; }
run ./build/rg_bk64 1370 3072 1024 50 && run ./build/rg_bk64_gm1 1370 3072 1024 50 && \
run ./build/rg_128x64 1280 1536 1024 50 && run ./build/rg_128x64_g4 1280 1536 1024 50 && \
bash tools/gpu_tasks.sh $O kern:t1370:--dim,1024,--heads,16,--batch,1,--tokens,1370,--only,N3072,--cold \
  kern:t1280:--dim,1024,--heads,16,--batch,1,--tokens,1280,--only,N3072,--cold \
  kern:t1024:--dim,1024,--heads,16,--batch,1,--tokens,1024,--only,N3072,--cold \
  kern:t2048:--dim,1024,--heads,16,--batch,1,--tokens,2048,--only,N3072,--cold \
  kern:f1024:--dim,1024,--heads,16,--batch,1,--tokens,1024,--only,fc1,--cold

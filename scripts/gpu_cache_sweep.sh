#!/bin/bash
# Hot-row replica cache sweep: 2 ranks sharing the box's GPU, DLRM 30 tables x ROWS rows sharded by table,
# peer exchange, a non-repeating request stream (--stream-pool distinct requests per rank), cache capacity
# per rank in CACHES (-1: auto, a quarter of the free device memory), REFRESH_S > 0: the background refresher
# runs while the clock does; STEPS (default 100) timed steps. One line per run -> gpurun_out/cache_sweep.jsonl.
# Round 6: every JSON line carries the exact top-k oracle of the served pool (hot_row_cache.oracle).
set -o pipefail
mkdir -p gpurun_out
export DTFS_SHARE_GPU=1 DTFS_HANG_DUMP_S=${HANG:-200}
: > gpurun_out/cache_sweep.jsonl
for spec in ${CACHES:-1048576:0 8388608:0 67108864:0 -1:0 -1:0.5}; do
  c=${spec%%:*}; r=${spec#*:}
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port 29621 bench.py --gpus 2 --model dlrm --table-rows ${ROWS:-20000000} --exchange peer --steps ${STEPS:-100} \
    --warmup 20 --requests-per-gpu 16 --qps 0 --qps-sweep= --stream-pool ${POOL:-4096} --hot-cache-rows $c \
    --cache-refresh-s $r > gpurun_out/cache_sweep_${c}_${r}.log 2>&1 \
    || { echo "cache $c refresh $r failed"; grep -v amdgpu.ids gpurun_out/cache_sweep_${c}_${r}.log | tail -40; exit 1; }
  grep '^{"metric' gpurun_out/cache_sweep_${c}_${r}.log >> gpurun_out/cache_sweep.jsonl
  echo "cache $c refresh $r: $(grep '^{"metric' gpurun_out/cache_sweep_${c}_${r}.log | cut -c1-200)"
done

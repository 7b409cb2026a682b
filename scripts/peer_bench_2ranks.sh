# 2 ranks sharing the box's GPU: DLRM with sharded tables, peer exchange vs RCCL all-to-all.
# ROWS (table rows), HANG (stack dump after that many seconds) override the defaults.
set -o pipefail
mkdir -p gpurun_out
export DTFS_SHARE_GPU=1 DTFS_HANG_DUMP_S=${HANG:-150}
for ex in ${EXCHANGES:-peer alltoall}; do
  timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --model dlrm --table-rows ${ROWS:-20000000} --exchange $ex --steps 100 --warmup 20 --requests-per-gpu 16 --qps 0 \
    > gpurun_out/peer_bench_$ex.log 2>&1 || { echo "bench $ex failed"; grep -v amdgpu.ids gpurun_out/peer_bench_$ex.log | tail -60; exit 1; }
  grep '^{"metric' gpurun_out/peer_bench_$ex.log | cut -c1-3000
done

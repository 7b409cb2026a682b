set -o pipefail
mkdir -p gpurun_out
export DTFS_SHARE_GPU=1
for ex in peer alltoall; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --model dlrm --table-rows 20000000 --exchange $ex --steps 100 --warmup 20 --requests-per-gpu 16 --qps 0 \
    > gpurun_out/peer_bench_$ex.log 2>&1 || { echo "bench $ex failed"; tail -30 gpurun_out/peer_bench_$ex.log; exit 1; }
  grep '^{"metric' gpurun_out/peer_bench_$ex.log | cut -c1-3000
done

set -o pipefail
export DTFS_SHARE_GPU=1 DTFS_HOST_THREADS=2
mkdir -p gpurun_out
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 -m tools.studies.peer_exchange --iters 300 > gpurun_out/peer_x2.log 2>&1 || { tail -30 gpurun_out/peer_x2.log; exit 1; }
grep '^{' gpurun_out/peer_x2.log
for pc in 0 262144 0 262144; do
 for mode in alltoall scatter; do
  DTFS_PEER_COMM=$pc timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 200 --warmup 20 --requests-per-gpu 1 --request-rows 512 --mode $mode --pool 8 --client-threads 2 --qps 0 --step-timeout-s 20 > gpurun_out/peer_bench_${mode}_${pc}.log 2>&1 || { tail -30 gpurun_out/peer_bench_${mode}_${pc}.log; exit 1; }
  echo "peer=$pc mode=$mode"; grep '^{' gpurun_out/peer_bench_${mode}_${pc}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('p50_request_ms'), d['config']['parallelism'])"
 done
done

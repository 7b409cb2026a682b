#!/bin/bash
# 8-rank rehearsal on ONE MI355X (DTFS_SHARE_GPU=1: every rank its own RCCL host id, RCCL over sockets):
# the code paths an 8-GPU node runs - alltoall fan-out, shared-arena scatter, sharded DLRM with the peer
# exchange - at world 8, with scaled-down steps (8 processes time-share the one GPU; rates are not xGMI numbers).
#   SETS="a2a;scatter;dlrm;dcnv2" bash scripts/gpu_rehearsal8.sh
# REF=1 then runs the reference's own topology: bench.py --reference-workload on 3 ranks sharing the GPU
# (scatter: 1,500 candidates split over 3 GPUs, 6 closed-loop clients) and the 1-GPU --over-grpc form.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp DTFS_SHARE_GPU=1 DTFS_HOST_THREADS=2 DTFS_HANG_DUMP_S=250
N=${N:-8}
common="--gpus $N --steps 30 --warmup 5 --prime-steps 20 --client-threads 2 --qps 400 --qps-seconds 0.5 --qps-sweep= --step-timeout-s 60"
port=$((29500 + RANDOM % 1000))
IFS=';' read -ra SETS <<< "${SETS:-a2a;scatter;dlrm}"
for s in "${SETS[@]}"; do
  case $s in
    a2a) args="--mode alltoall --requests-per-gpu 8 --request-rows 256 --pool 8 --small-buckets 256";;
    scatter) args="--mode scatter --requests-per-gpu 8 --request-rows 256 --pool 8 --small-buckets 256";;
    dlrm) args="--model dlrm --exchange peer --table-rows 2000000 --requests-per-gpu 8 --request-rows 256 --stream-pool 64 --small-buckets 256 --cache-learn-rounds 2";;
    dcnv2) args="--model dcn_v2 --mode alltoall --requests-per-gpu 8 --request-rows 256 --pool 8 --small-buckets 256";;
    *) echo "unknown set $s"; exit 2;;
  esac
  port=$((port + 1))
  timeout -k 10 ${SET_TIMEOUT:-300} python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=$N --master-addr 127.0.0.1 \
    --master-port $port bench.py $common $args > gpurun_out/rehearsal8_$s.log 2>&1 \
    || { echo "rehearsal $s failed"; tail -40 gpurun_out/rehearsal8_$s.log; exit 1; }
  echo "[$s]"; grep '^{"metric' gpurun_out/rehearsal8_$s.log | cut -c1-3000
done
if [ "${REF:-0}" = "1" ]; then
  port=$((port + 1))
  timeout -k 10 ${SET_TIMEOUT:-300} python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 3 --reference-workload --ref-requests ${REF_REQUESTS:-300} \
    > gpurun_out/reference3.log 2>&1 || { echo "reference workload at 3 ranks failed"; tail -40 gpurun_out/reference3.log; exit 1; }
  echo "[reference 3 ranks]"; grep -E '^Average|^\{' gpurun_out/reference3.log | cut -c1-2000
  unset DTFS_SHARE_GPU
  timeout -k 10 ${SET_TIMEOUT:-300} python -u bench.py --reference-workload --over-grpc --ref-requests ${REF_REQUESTS:-1000} \
    > gpurun_out/reference_grpc.log 2>&1 || { echo "reference workload over gRPC failed"; tail -40 gpurun_out/reference_grpc.log; exit 1; }
  echo "[reference over gRPC, 1 GPU]"; grep -E '^Average|^\{' gpurun_out/reference_grpc.log | cut -c1-2000
fi
echo "rehearsal8 done"

#!/bin/bash
# gRPC front door on one MI355X: throughput ceiling (client processes x threads,
# bench/grpc_ceiling.py), then the reference closed-loop workload and the
# fixed-QPS sweep (scripts/gpu_qps.sh). Results under gpurun_out/grpc/.
set -o pipefail
mkdir -p gpurun_out/grpc
export TMPDIR=/tmp
timeout -k 10 240 python -u -m distributed_tf_serving_amd.bench.grpc_ceiling --preset deepfm_1gpu \
  --procs ${PROCS:-1 2 4} --threads 16 --seconds 5 --out gpurun_out/grpc/ceiling_raw.json \
  > gpurun_out/grpc/ceiling_raw.log 2>&1 || { echo "ceiling raw failed"; tail -20 gpurun_out/grpc/ceiling_raw.log; exit 1; }
grep '^{' gpurun_out/grpc/ceiling_raw.log
if [ "${PACKED:-1}" = 1 ]; then
  timeout -k 10 240 python -u -m distributed_tf_serving_amd.bench.grpc_ceiling --preset deepfm_1gpu --packed \
    --procs ${PROCS:-1 2 4} --threads 16 --seconds 5 --out gpurun_out/grpc/ceiling_packed.json \
    > gpurun_out/grpc/ceiling_packed.log 2>&1 || { echo "ceiling packed failed"; tail -20 gpurun_out/grpc/ceiling_packed.log; exit 1; }
  grep '^{' gpurun_out/grpc/ceiling_packed.log
fi
if [ "${QPS_SWEEP:-1}" = 1 ]; then
  CLOSED_LOOP=1 bash scripts/gpu_qps.sh && SKIP_DCN=1 bash scripts/gpu_qps.sh
fi

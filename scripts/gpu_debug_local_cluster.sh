#!/bin/bash
# debug: the config-4 local cluster worker on 2 ranks sharing the GPU, full logs (faulthandler on)
set -o pipefail
mkdir -p gpurun_out/dbg
export DTFS_SHARE_GPU=1 DTFS_HOST_THREADS=2 DTFS_HANG_DUMP_S=100 PYTHONFAULTHANDLER=1
timeout -k 10 150 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port 29731 --log-dir gpurun_out/dbg/tr --redirects 3 --tee 3 tests/cluster_worker.py --mode local --preset dlrm --grpc-port 29800 \
  --out gpurun_out/dbg > gpurun_out/dbg/run.log 2>&1
echo "rc=$?"
tail -50 gpurun_out/dbg/run.log
find gpurun_out/dbg -name "*.log" -path "*tr*" | head

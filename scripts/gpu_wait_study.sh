#!/bin/bash
# Cross-stream wait cost study + GEMM variants vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/wait
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/wait -o run --output-format rocpd -- python3 -m distributed_tf_serving_amd.bench.wait_gap > gpurun_out/wait.log 2>&1 || { echo "wait study failed"; tail -30 gpurun_out/wait.log; exit 1; }
db=$(find gpurun_out/wait -name '*.db' | head -1)
python -m distributed_tf_serving_amd.bench.wait_gap --analyze "$db" | tee gpurun_out/wait_summary.txt
timeout -k 10 300 python -u -m distributed_tf_serving_amd.bench.microbench --gemm-variants > gpurun_out/gemm_variants.log 2>&1 || { echo "gemm variants failed"; tail -30 gpurun_out/gemm_variants.log; exit 1; }
cat gpurun_out/gemm_variants.log

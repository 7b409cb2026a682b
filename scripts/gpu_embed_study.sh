#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m distributed_tf_serving_amd.bench.microbench --embed-study > gpurun_out/embed_study.log 2>&1 || { tail -30 gpurun_out/embed_study.log; exit 1; }
cat gpurun_out/embed_study.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "embed" -d gpurun_out/pmc_fetch -o run -- python3 -m distributed_tf_serving_amd.bench.microbench --embed-study > gpurun_out/pmc1.log 2>&1 || { tail -30 gpurun_out/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-include-regex "embed" -d gpurun_out/pmc_write -o run -- python3 -m distributed_tf_serving_amd.bench.microbench --embed-study > gpurun_out/pmc2.log 2>&1 || { tail -30 gpurun_out/pmc2.log; exit 1; }
find gpurun_out/pmc_fetch gpurun_out/pmc_write -type f | head

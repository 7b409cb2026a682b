#!/bin/bash
# Kernel tests for the new paths first, then the full GPU suite, microbench studies, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "tail or pipelined or full_mlp or embed" > gpurun_out/pytest_new.log 2>&1 || { echo "new kernel tests failed"; tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -2 gpurun_out/pytest_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -m distributed_tf_serving_amd.bench.microbench --tail-study > gpurun_out/tail_study.log 2>&1 || { tail -20 gpurun_out/tail_study.log; exit 1; }
cat gpurun_out/tail_study.log | grep op
timeout -k 10 200 python -u -m distributed_tf_serving_amd.bench.microbench --embed-study > gpurun_out/embed_study.log 2>&1 || { tail -20 gpurun_out/embed_study.log; exit 1; }
grep op gpurun_out/embed_study.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log

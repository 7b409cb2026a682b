#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for args in "" "--force-fanout" ""; do
  timeout -k 10 200 python -u bench.py $args > gpurun_out/bench_c.log 2>&1 || { echo "bench $args failed"; tail -20 gpurun_out/bench_c.log; exit 1; }
  echo "bench $args: $(grep metric gpurun_out/bench_c.log)"
done

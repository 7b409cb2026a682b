#!/bin/bash
# One GPU call: gpu tests, smoke, 1-GPU bench, then a kernel-trace profile of
# the bench. Each step has its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o run --output-format rocpd -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof.log; exit 1; }
db=$(find gpurun_out/prof -name '*.db' | head -1)
python -m distributed_tf_serving_amd.bench.prof_summary "$db" --steps 110 --title "bench.py default (DeepFM, 32 x 512-candidate requests = 16384 rows/step), 1 MI355X" > gpurun_out/prof_summary.md && cat gpurun_out/prof_summary.md

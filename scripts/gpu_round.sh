#!/bin/bash
# One GPU call: GPU tests (optionally a subset), smoke, bench, kernel profile.
#   TESTS="tests/test_live_gpu.py" BENCH_ARGS="--steps 200" PROFILE=1 bash scripts/gpu_round.sh
# Each step runs under its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "${SKIP_SMOKE:-0}" != "1" ]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log | grep -v amdgpu.ids
fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py ${BENCH_ARGS:-} --json-extra > gpurun_out/bench.log 2>&1 \
  || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -4
if [ "${PROFILE:-0}" = "1" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof -o run --output-format rocpd \
    -- python3 bench.py ${PROF_ARGS:---steps 100 --warmup 10 --qps 0} > gpurun_out/prof.log 2>&1 \
    || { echo "prof failed"; tail -30 gpurun_out/prof.log; exit 1; }
  db=$(find gpurun_out/prof -name '*.db' | head -1)
  python -m tools.prof_summary "$db" --steps ${PROF_STEPS:-110} \
    --title "${PROF_TITLE:-bench.py live path (DeepFM, 32 x 512-candidate requests per step), 1 MI355X}" \
    > gpurun_out/prof_summary.md && cat gpurun_out/prof_summary.md
fi

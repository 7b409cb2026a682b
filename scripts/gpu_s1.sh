#!/bin/bash
# session GPU step: targeted tests, a kernel study, optional benches; stops at the first failure
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_s1.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_s1.log; exit 1; }
  tail -3 gpurun_out/pytest_s1.log
fi
if [ -n "${STUDY:-}" ]; then
  timeout -k 10 300 python -u -m $STUDY > gpurun_out/study.log 2>&1 || { echo "study failed"; tail -30 gpurun_out/study.log; exit 1; }
  cat gpurun_out/study.log
fi
for m in ${MODELS:-}; do
  timeout -k 10 300 python -u bench.py --model $m --steps ${STEPS:-200} --warmup 20 \
    > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -40 gpurun_out/bench_$m.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['value']/1e6, 'M', d['ms_per_step'], 'ms', d.get('fp32_check'), 'fixed_qps p50', d.get('p50_at_fixed_qps_ms'))"
done

#!/bin/bash
# Interleaved A/B of an environment toggle on the served bench: AB_VAR=NAME AB_VALUES="0 1" ROUNDS=2 MODEL=deepfm
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-400} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $AB_VALUES; do
    for m in ${MODEL:-deepfm}; do
      env $AB_VAR=$v timeout -k 10 300 python -u bench.py --model $m --steps ${STEPS:-200} --warmup 20 \
        > gpurun_out/ab/${m}_${v}_$r.log 2>&1 || { echo "bench $m $v failed"; tail -30 gpurun_out/ab/${m}_${v}_$r.log; exit 1; }
      grep '^{"metric' gpurun_out/ab/${m}_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m $AB_VAR=$v round $r', round(d['value']/1e6,2), 'M', d['ms_per_step'], 'ms fp32', d['fp32_check'].get('max_abs_diff'), 'p50fq', d.get('p50_at_fixed_qps_ms'))"
    done
  done
done

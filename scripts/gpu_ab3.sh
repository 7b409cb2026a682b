#!/bin/bash
# Interleaved A/B of bench.py arms inside ONE GPU call (box-to-box spread is larger than most effects).
#   ARMS="--h2d-wait host|--h2d-wait device" MODEL=deepfm REPS=2 bash scripts/gpu_ab3.sh
set -o pipefail
mkdir -p gpurun_out/ab3
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/ab3/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ab3/pytest.log; exit 1; }
  tail -2 gpurun_out/ab3/pytest.log
fi
IFS='|' read -ra arms <<< "${ARMS:-}"
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for arm in "${arms[@]}"; do
    i=$((i + 1))
    log=gpurun_out/ab3/${MODEL:-deepfm}_arm${i}_rep${rep}.log
    timeout -k 10 240 python -u bench.py --model ${MODEL:-deepfm} --steps ${STEPS:-200} --warmup 20 --qps 0 $arm \
      > $log 2>&1 || { echo "arm '$arm' failed"; tail -30 $log; exit 1; }
    grep '^{"metric' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rep", '$rep', "arm", repr("""'"$arm"'"""), round(d["value"]/1e6,2), "M", d["ms_per_step"], "ms/step", d.get("fp32_check",{}).get("max_abs_diff"))'
  done
done

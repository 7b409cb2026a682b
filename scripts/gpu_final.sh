#!/bin/bash
# Round-end evidence in one call: GPU tests, smoke, 200-step bench + kernel profile (scripts/gpu_round.sh),
# then the driver's short form (--steps 20 --warmup 5) REPS times, fresh process each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_ROUND:-0}" != "1" ]; then
  BENCH_ARGS="--steps 200 --warmup 20" PROFILE=${PROFILE:-1} bash scripts/gpu_round.sh || exit 1
fi
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${SHORT_ARGS:-} > gpurun_out/bench20_$i.log 2>&1 \
    || { tail -20 gpurun_out/bench20_$i.log; exit 1; }
  grep '^{"metric' gpurun_out/bench20_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("20-step", round(d["value"]/1e6,2), d["ms_per_step"], "prime", d.get("prime_steps"))'
done

#!/bin/bash
# bench.py under each step-done signalling mode (csrc/runtime/step_runner.cpp)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 0 1 2 3; do
  DTFS_EVENT_MODE=$m timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 > gpurun_out/bench_ev$m.log 2>&1 || { echo "mode $m failed"; tail -20 gpurun_out/bench_ev$m.log; exit 1; }
  echo "mode $m: $(grep metric gpurun_out/bench_ev$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))')"
done
for m in 0 3; do
  DTFS_EVENT_MODE=$m timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 --force-fanout > gpurun_out/bench_fan_ev$m.log 2>&1 || { echo "fanout mode $m failed"; tail -20 gpurun_out/bench_fan_ev$m.log; exit 1; }
  echo "fanout mode $m: $(grep metric gpurun_out/bench_fan_ev$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))')"
done

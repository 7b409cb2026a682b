#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "DTFS_H2D_STREAMS=2|" "DTFS_H2D_STREAMS=1|" "DTFS_H2D_STREAMS=3|" "DTFS_H2D_STREAMS=2|--force-fanout" "DTFS_H2D_STREAMS=1|--force-fanout" "DTFS_H2D_STREAMS=2|--requests-per-gpu 16"; do
  i=$((i+1)); envs=${cfg%%|*}; args=${cfg#*|}
  env $envs timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 $args > gpurun_out/bench_s$i.log 2>&1 || { echo "$cfg failed"; tail -20 gpurun_out/bench_s$i.log; exit 1; }
  echo "$cfg: $(grep metric gpurun_out/bench_s$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))')"
done

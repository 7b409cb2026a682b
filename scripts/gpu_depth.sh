#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for cfg in "DTFS_SPIN_WAIT=0|--slots 4" "DTFS_SPIN_WAIT=1|--slots 4" "DTFS_SPIN_WAIT=0|--slots 5" "DTFS_SPIN_WAIT=0|--slots 6" "DTFS_SPIN_WAIT=1|--slots 6" "DTFS_H2D_STREAMS=1|--slots 6"; do
  i=$((i+1)); envs=${cfg%%|*}; args=${cfg#*|}
  env $envs timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 --json-extra $args > gpurun_out/bench_d$i.log 2>&1 || { echo "$cfg failed"; tail -20 gpurun_out/bench_d$i.log; exit 1; }
  echo "$cfg: $(grep metric gpurun_out/bench_d$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))') $(grep host_phase gpurun_out/bench_d$i.log)"
done

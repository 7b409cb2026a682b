#!/bin/bash
# Interleaved A/B of bench.py configurations in ONE GPU call (same box, same
# clocks; cdna_hip_programming.md rule 24: never compare across boxes).
#   CONFIGS="chain|DTFS_MX_CHAIN=1|--model dcn_v2;nochain|DTFS_MX_CHAIN=0|--model dcn_v2" ROUNDS=2 \
#     bash scripts/gpu_ab.sh
# Each config is "name|ENV=V ENV2=V2|bench args"; BENCH_ARGS are common to all.
# One line per run: name round scores/s ms_per_step p50_request_ms. Logs: gpurun_out/ab/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
IFS=';' read -ra CFGS <<< "${CONFIGS:?set CONFIGS}"
for round in $(seq 1 ${ROUNDS:-2}); do
  for cfg in "${CFGS[@]}"; do
    name=${cfg%%|*}; rest=${cfg#*|}; envs=${rest%%|*}; args=${rest#*|}
    log=gpurun_out/ab/${name}_r$round.log
    env $envs timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py ${BENCH_ARGS:---steps 200 --warmup 20 --qps 0} $args \
      > $log 2>&1 || { echo "$name failed"; tail -20 $log; exit 1; }
    echo "$name $round $(grep '^{"metric' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6, 2), d["ms_per_step"], d.get("p50_request_ms"))')"
  done
done

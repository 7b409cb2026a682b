#!/bin/bash
# bench.py under H2D variants (csrc/runtime/step_runner.cpp: DTFS_COPY_WAIT, DTFS_H2D_SPLIT)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for envs in "DTFS_COPY_WAIT=1" "DTFS_COPY_WAIT=0" "DTFS_H2D_SPLIT=2" "DTFS_H2D_SPLIT=3" "DTFS_H2D_SPLIT=2 DTFS_COPY_WAIT=1"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python -u bench.py --steps 400 --warmup 40 > gpurun_out/bench_h2d$i.log 2>&1 || { echo "$envs failed"; tail -20 gpurun_out/bench_h2d$i.log; exit 1; }
  echo "$envs: $(grep metric gpurun_out/bench_h2d$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))')"
done
rm -rf gpurun_out/prof_h2d
DTFS_H2D_SPLIT=2 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/prof_h2d -o run --output-format rocpd -- python3 bench.py --steps 100 --warmup 10 > gpurun_out/prof_h2d.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_h2d.log; exit 1; }

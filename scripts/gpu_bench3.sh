#!/bin/bash
# Three back-to-back default bench runs (box-noise check).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py > gpurun_out/b$i.log 2>&1 || { echo "bench $i failed"; tail -20 gpurun_out/b$i.log; exit 1; }
  grep '^{' gpurun_out/b$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_request_ms"], d["p99_request_ms"])'
done

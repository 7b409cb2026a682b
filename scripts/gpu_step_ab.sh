#!/bin/bash
# Interleaved A/B of step-level knobs on one box (box-to-box spread is large):
# event modes (how "step done" is signalled) and the embedding-gather study.
set -o pipefail
mkdir -p gpurun_out/stepab
export TMPDIR=/tmp
timeout -k 10 200 python -u -m distributed_tf_serving_amd.bench.microbench --embed-study > gpurun_out/stepab/embed_study.jsonl 2>&1 || { echo "embed study failed"; tail -5 gpurun_out/stepab/embed_study.jsonl; exit 1; }
grep '^{' gpurun_out/stepab/embed_study.jsonl
for round in 1 2; do
  for m in ${MODES:-0 2 3}; do
    DTFS_EVENT_MODE=$m timeout -k 10 200 python -u bench.py --steps 300 --warmup 30 --qps 0 > gpurun_out/stepab/ev${m}_r$round.log 2>&1 || { echo "mode $m failed"; tail -20 gpurun_out/stepab/ev${m}_r$round.log; exit 1; }
    echo "mode $m round $round: $(grep '^{"metric' gpurun_out/stepab/ev${m}_r$round.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), d["ms_per_step"], d.get("fp32_check",{}).get("status"))')"
  done
done

#!/bin/bash
# bench.py for the other BASELINE configs on one MI355X (live path), with a
# kernel profile of each: DCN-v2 fp8 (config 5), DLRM (config 4, tables
# shrunk to fit one GPU), DCN (the reference's model).
set -o pipefail
mkdir -p gpurun_out/models
export TMPDIR=/tmp
for m in ${MODELS:-dcn_v2 dlrm dcn}; do
  timeout -k 10 400 python -u bench.py --model $m --steps ${STEPS:-100} --warmup 10 --qps 0 --json-extra > gpurun_out/models/$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/models/$m.log; exit 1; }
  grep '^{"metric' gpurun_out/models/$m.log | cut -c1-700
  if [ "${PROFILE:-1}" = 1 ]; then
    rm -rf gpurun_out/models/prof_$m
    timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/models/prof_$m -o run --output-format rocpd \
      -- python3 bench.py --model $m --steps 40 --warmup 5 --qps 0 > gpurun_out/models/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -10 gpurun_out/models/prof_$m.log; exit 1; }
    db=$(find gpurun_out/models/prof_$m -name '*.db' | head -1)
    python -m distributed_tf_serving_amd.bench.prof_summary "$db" --steps 45 --title "bench.py --model $m (live path), 1 MI355X" > gpurun_out/models/prof_$m.md && head -16 gpurun_out/models/prof_$m.md
  fi
done

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_native_fanout_gpu.py -x -q --timeout 120 --timeout-method thread -k "arena or varint or serving_loop or fanout" > gpurun_out/pytest_varint.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_varint.log; exit 1; }
tail -2 gpurun_out/pytest_varint.log
for args in "--encoding packed" "" "--encoding packed --force-fanout"; do
  timeout -k 10 200 python -u bench.py $args --json-extra > gpurun_out/bench_v.log 2>&1 || { echo "bench $args failed"; tail -20 gpurun_out/bench_v.log; exit 1; }
  echo "bench $args: $(grep metric gpurun_out/bench_v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_request_ms"], d.get("score_check"))') $(grep host_phase gpurun_out/bench_v.log)"
done
rm -rf gpurun_out/prof_v
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_v -o run --output-format rocpd -- python3 bench.py --encoding packed --steps 100 --warmup 10 > gpurun_out/prof_v.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_v.log; exit 1; }
db=$(find gpurun_out/prof_v -name '*.db' | head -1)
python -m distributed_tf_serving_amd.bench.prof_summary "$db" --steps 110 --title "bench.py --encoding packed (DeepFM, 32 x 512-candidate packed-varint requests = 16384 rows/step), 1 MI355X" > gpurun_out/prof_v_summary.md && cat gpurun_out/prof_v_summary.md

set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_live_gpu.py tests/test_kernels_gpu.py tests/test_native_fanout_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -2 gpurun_out/ab/pytest.log
for cfg in "narrow_gate::" "raw_gate:--no-narrow:" "narrow_nogate::DTFS_H2D_GATE=0" "raw_nogate:--no-narrow:DTFS_H2D_GATE=0"; do
  name=${cfg%%:*}; rest=${cfg#*:}; args=${rest%%:*}; envs=${rest#*:}
  env $envs timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --qps 0 $args --json-extra > gpurun_out/ab/$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/ab/$name.log; exit 1; }
  echo "$name: $(grep '^{"metric' gpurun_out/ab/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"]/1e6, d["ms_per_step"], d["p50_request_ms"])')"
done

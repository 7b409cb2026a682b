#!/bin/bash
# Round-3 evidence in one GPU call: GPU tests, smoke, DeepFM / DCN / reference-workload benches, DeepFM
# kernel profile. Each step under its own time limit; the script stops at the first failure.
#   SKIP_TESTS=1 MODELS="deepfm dcn" PROFILE=1 bash scripts/gpu_r3.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/smoke.log
fi
for m in ${MODELS:-deepfm}; do
  timeout -k 10 300 python -u bench.py --model $m --steps ${STEPS:-200} --warmup 20 --json-extra \
    > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -40 gpurun_out/bench_$m.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$m.log
done
if [ "${REF:-0}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --reference-workload > gpurun_out/bench_ref.log 2>&1 \
    || { echo "reference workload failed"; tail -30 gpurun_out/bench_ref.log; exit 1; }
  grep -E '^Average|^\{' gpurun_out/bench_ref.log
fi
if [ "${FRONTENDS:-}" != "" ]; then
  # the reference workload (DCN, 1500 identical candidates, 6 closed-loop clients) over the gRPC front door,
  # with K server processes sharing the port (serving/server.py --frontends K)
  mkdir -p gpurun_out/frontends
  for k in $FRONTENDS; do
    port=$((9950 + k))
    timeout -k 10 400 python -u -m distributed_tf_serving_amd.serving.server --preset reference_dcn --port $port --frontends $k \
      > gpurun_out/frontends/server_$k.log 2>&1 &
    spid=$!
    python - "$port" <<'PYEOF' || { echo "server $k did not start"; kill $spid; tail -20 gpurun_out/frontends/server_$k.log; exit 1; }
import socket, sys, time
port = int(sys.argv[1]); t0 = time.time()
while time.time() - t0 < 200:
    try:
        socket.create_connection(("127.0.0.1", port), timeout=1).close(); sys.exit(0)
    except OSError:
        time.sleep(1)
sys.exit(1)
PYEOF
    sleep $((3 * k))
    timeout -k 10 200 python -u -m distributed_tf_serving_amd.client.loadgen --hosts 127.0.0.1:$port --backends 1 \
      --candidates 1500 --id-mode reference --concurrency 6 --requests ${REF_REQS:-1000} --warmup 30 --quiet \
      --json-out gpurun_out/frontends/ref_grpc_$k.json > gpurun_out/frontends/loadgen_$k.log 2>&1
    rc=$?
    kill $spid; wait $spid 2>/dev/null
    [ $rc = 0 ] || { echo "loadgen $k failed"; tail -20 gpurun_out/frontends/loadgen_$k.log; exit 1; }
    echo "frontends=$k $(grep Average gpurun_out/frontends/loadgen_$k.log) $(cat gpurun_out/frontends/ref_grpc_$k.json)"
  done
fi
if [ "${PROFILE:-0}" = "1" ]; then
  for pm in ${PROF_MODELS:-deepfm}; do
    rm -rf gpurun_out/prof_$pm
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_$pm -o run --output-format rocpd \
      -- python3 bench.py --model $pm --steps 100 --warmup 10 --qps 0 > gpurun_out/prof_$pm.log 2>&1 \
      || { echo "prof $pm failed"; tail -30 gpurun_out/prof_$pm.log; exit 1; }
    db=$(find gpurun_out/prof_$pm -name '*.db' | head -1)
    case $pm in deepfm|wdl|dcn) sk="gemm_gather --min-us 80";; dlrm) sk="bottom_mlp3 --min-us 14";; *) sk="embed_pipe --min-us 30";; esac
    python -m tools.prof_summary "$db" --steps ${PROF_STEPS:-110} --step-kernel $sk \
      --title "bench.py live path ($pm, default step shape), 1 MI355X" > gpurun_out/prof_summary_$pm.md \
      && head -30 gpurun_out/prof_summary_$pm.md
  done
fi

#!/bin/bash
# Open-loop latency at fixed offered load (BASELINE.json: "p50 request latency
# at fixed QPS") through the gRPC front door on one MI355X.
#   preset deepfm_1gpu : BASELINE config 2 (DeepFM 1Mx64, 512-candidate requests, zipf ids)
#   preset reference_dcn: the reference workload shape (DCN, 1500 candidates, ids 1..43)
# Each server is started in the background and stopped by its own PID.
set -u
mkdir -p gpurun_out/qps
OUT=gpurun_out/qps

wait_port() {  # bounded wait for the server to accept connections
  python - "$1" <<'EOF'
import socket, sys, time
port = int(sys.argv[1]); t0 = time.time()
while time.time() - t0 < 150:
    try:
        socket.create_connection(("127.0.0.1", port), timeout=1).close(); sys.exit(0)
    except OSError:
        time.sleep(1)
sys.exit(1)
EOF
}

run_preset() {  # preset port candidates id_mode qps...
  local preset=$1 port=$2 cand=$3 idm=$4; shift 4
  timeout -k 10 400 python -u -m distributed_tf_serving_amd.serving.server --preset "$preset" --port "$port" --grpc-workers "${GRPC_WORKERS:-32}" \
      > "$OUT/server_$preset.log" 2>&1 &
  local spid=$!
  if ! wait_port "$port"; then echo "server $preset did not come up"; kill "$spid"; return 1; fi
  local rc=0
  for q in "$@"; do
    timeout -k 10 90 python -u -m distributed_tf_serving_amd.client.loadgen --hosts "127.0.0.1:$port" \
        --backends 1 --candidates "$cand" --id-mode "$idm" --raw-tensors --qps "$q" --requests 2000 \
        --concurrency 1 --warmup 200 --quiet --json-out "$OUT/${preset}_qps$q.json" \
        > "$OUT/loadgen_${preset}_$q.log" 2>&1 || { rc=$?; echo "loadgen $preset $q rc=$rc"; break; }
    cat "$OUT/${preset}_qps$q.json"; echo
  done
  kill "$spid"; wait "$spid" 2>/dev/null
  return $rc
}


# the reference's own closed-loop shape (6 clients x 1000 requests, DCNClient.java:205-241), one backend
if [ "${CLOSED_LOOP:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m distributed_tf_serving_amd.serving.server --preset reference_dcn --port 9997 \
      > "$OUT/server_closed.log" 2>&1 &
  spid=$!
  wait_port 9997 && timeout -k 10 120 python -u -m distributed_tf_serving_amd.client.loadgen \
      --hosts 127.0.0.1:9997 --backends 1 --candidates 1500 --id-mode reference --quiet \
      --json-out "$OUT/reference_closed_loop.json" > "$OUT/loadgen_closed.log" 2>&1
  rc=$?
  kill "$spid"; wait "$spid" 2>/dev/null
  cat "$OUT/reference_closed_loop.json"; echo
  exit $rc
fi

run_preset deepfm_1gpu 9999 512 zipf ${DEEPFM_QPS:-250 500 1000 2000} && \
{ [ "${SKIP_DCN:-0}" = 1 ] || run_preset reference_dcn 9998 1500 reference 250 500 1000; }

#!/bin/bash
# Measurement studies on one MI355X, one per GPU call:
#   bash scripts/gpu_study.sh counters   rocprofv3 --pmc passes over the serving-shape forwards
#                                        + hipBLASLt comparison        -> gpurun_out/ctr/
#   bash scripts/gpu_study.sh models     bench.py + kernel profile per model (MODELS="dcn_v2 dlrm dcn")
#   bash scripts/gpu_study.sh grpc       gRPC front-door ceiling (client procs x threads) + qps
#   bash scripts/gpu_study.sh qps        fixed-QPS open loop over gRPC (+ CLOSED_LOOP=1: reference workload)
#   bash scripts/gpu_study.sh trace      roctx + kernel + copy timeline of the live bench (ARGS=...)
#   bash scripts/gpu_study.sh embed      embedding-gather study + its counters
#   bash scripts/gpu_study.sh gemm       GEMM tile-variant sweep + MX-fp8 cross-layer forms
# Every GPU step runs under its own time limit; the script stops at the first failure.
# Counter budget per --pmc pass (MI355X): <= 8 SQ, <= 4 TCC (FETCH_SIZE = 3, WRITE_SIZE = 2), <= 2 GRBM.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

counters() {
  local OUT=gpurun_out/ctr
  rm -rf $OUT && mkdir -p $OUT
  local PASS_SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  local PASS_FETCH="FETCH_SIZE GRBM_GUI_ACTIVE"
  local PASS_WRITE="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  for model in ${MODELS:-deepfm dcn_v2}; do
    local rows=16384; [ $model = dcn_v2 ] && rows=8192
    local i=0
    for pass in "$PASS_SQ" "$PASS_FETCH" "$PASS_WRITE"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/${model}_p$i -o run \
        -- python3 -m tools.studies.kernel_drive --model $model --rows $rows --iters 10 \
        > $OUT/${model}_p$i.log 2>&1 || { echo "pass $i of $model failed"; tail -5 $OUT/${model}_p$i.log; return 1; }
    done
    mkdir -p $OUT/sum_$model && cp -r $OUT/${model}_p* $OUT/sum_$model/ 2>/dev/null
    python -m tools.counters_summary $OUT/sum_$model \
      --title "$model serving-shape forward, 1 MI355X (rocprofv3 --pmc, 3 passes)" > $OUT/summary_$model.md
    cat $OUT/summary_$model.md
  done
  timeout -k 10 300 python -u -m tools.studies.microbench --serving > $OUT/microbench.jsonl 2>&1 \
    || { echo "microbench failed"; tail -5 $OUT/microbench.jsonl; return 1; }
  grep '^{' $OUT/microbench.jsonl
}

models() {
  mkdir -p gpurun_out/models
  for m in ${MODELS:-dcn_v2 dlrm dcn}; do
    timeout -k 10 400 python -u bench.py --model $m --steps ${STEPS:-100} --warmup 10 --qps 0 --json-extra \
      > gpurun_out/models/$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/models/$m.log; return 1; }
    grep '^{"metric' gpurun_out/models/$m.log | cut -c1-700
    if [ "${PROFILE:-1}" = 1 ]; then
      rm -rf gpurun_out/models/prof_$m
      timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/models/prof_$m -o run \
        --output-format rocpd -- python3 bench.py --model $m --steps 40 --warmup 5 --qps 0 \
        > gpurun_out/models/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -10 gpurun_out/models/prof_$m.log; return 1; }
      local db=$(find gpurun_out/models/prof_$m -name '*.db' | head -1)
      python -m tools.prof_summary "$db" --steps 45 \
        --title "bench.py --model $m (live path), 1 MI355X" > gpurun_out/models/prof_$m.md && head -16 gpurun_out/models/prof_$m.md
    fi
  done
}

wait_port() {  # bounded wait for a server to accept connections
  python - "$1" <<'PYEOF'
import socket, sys, time
port = int(sys.argv[1]); t0 = time.time()
while time.time() - t0 < 150:
    try:
        socket.create_connection(("127.0.0.1", port), timeout=1).close(); sys.exit(0)
    except OSError:
        time.sleep(1)
sys.exit(1)
PYEOF
}

qps_preset() {  # preset port candidates id_mode qps...  (server stopped by its own PID)
  local OUT=gpurun_out/qps preset=$1 port=$2 cand=$3 idm=$4; shift 4
  mkdir -p $OUT
  timeout -k 10 400 python -u -m distributed_tf_serving_amd.serving.server --preset "$preset" --port "$port" \
    --grpc-workers "${GRPC_WORKERS:-32}" > "$OUT/server_$preset.log" 2>&1 &
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

qps() {
  local OUT=gpurun_out/qps
  mkdir -p $OUT
  if [ "${CLOSED_LOOP:-0}" = 1 ]; then
    # the reference's own closed-loop shape (6 clients x 1000 requests, DCNClient.java:205-241), one backend
    timeout -k 10 300 python -u -m distributed_tf_serving_amd.serving.server --preset reference_dcn --port 9997 \
      > "$OUT/server_closed.log" 2>&1 &
    local spid=$!
    wait_port 9997 && timeout -k 10 120 python -u -m distributed_tf_serving_amd.client.loadgen \
      --hosts 127.0.0.1:9997 --backends 1 --candidates 1500 --id-mode reference --quiet \
      --json-out "$OUT/reference_closed_loop.json" > "$OUT/loadgen_closed.log" 2>&1
    local rc=$?
    kill "$spid"; wait "$spid" 2>/dev/null
    cat "$OUT/reference_closed_loop.json"; echo
    [ $rc = 0 ] || return $rc
  fi
  qps_preset deepfm_1gpu 9999 512 zipf ${DEEPFM_QPS:-250 500 1000 2000} && \
    { [ "${SKIP_DCN:-0}" = 1 ] || qps_preset reference_dcn 9998 1500 reference 250 500 1000; }
}

grpc() {
  mkdir -p gpurun_out/grpc
  for enc in raw packed; do
    [ $enc = packed ] && [ "${PACKED:-1}" != 1 ] && continue
    local flag=""; [ $enc = packed ] && flag=--packed
    timeout -k 10 240 python -u -m tools.studies.grpc_ceiling --preset ${PRESET:-deepfm_1gpu} $flag \
      --procs ${PROCS:-1 2 4} --threads 16 --seconds 5 --frontends ${FRONTENDS:-1} --out gpurun_out/grpc/ceiling_$enc.json \
      > gpurun_out/grpc/ceiling_$enc.log 2>&1 || { echo "ceiling $enc failed"; tail -20 gpurun_out/grpc/ceiling_$enc.log; return 1; }
    grep '^{' gpurun_out/grpc/ceiling_$enc.log
  done
  if [ "${QPS_SWEEP:-1}" = 1 ]; then
    CLOSED_LOOP=1 SKIP_DCN=1 qps
  fi
}

trace() {
  export DTFS_TRACE=1
  rm -rf gpurun_out/tl && mkdir -p gpurun_out/tl
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format rocpd -d gpurun_out/tl -o run \
    -- python3 bench.py --steps 60 --warmup 10 --qps 0 ${ARGS:-} > gpurun_out/tl/bench.log 2>&1 \
    || { echo "trace failed"; tail -20 gpurun_out/tl/bench.log; return 1; }
  grep '^{"metric' gpurun_out/tl/bench.log | cut -c1-300
}

embed() {
  timeout -k 10 200 python -u -m tools.studies.microbench --embed-study > gpurun_out/embed_study.log 2>&1 \
    || { tail -30 gpurun_out/embed_study.log; return 1; }
  grep '^{' gpurun_out/embed_study.log
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "embed" -d gpurun_out/pmc_fetch \
    -o run -- python3 -m tools.studies.microbench --embed-study > gpurun_out/pmc1.log 2>&1 \
    || { tail -30 gpurun_out/pmc1.log; return 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    --kernel-include-regex "embed" -d gpurun_out/pmc_write -o run -- python3 -m tools.studies.microbench \
    --embed-study > gpurun_out/pmc2.log 2>&1 || { tail -30 gpurun_out/pmc2.log; return 1; }
}

gemm() {
  timeout -k 10 300 python -u -m tools.studies.microbench --gemm-variants > gpurun_out/gemm_variants.log 2>&1 \
    || { echo "gemm variants failed"; tail -30 gpurun_out/gemm_variants.log; return 1; }
  grep '^{' gpurun_out/gemm_variants.log
  timeout -k 10 200 python -u -m tools.studies.mx_ab ${MX_ROWS:-16384} > gpurun_out/mx_ab.log 2>&1 \
    || { echo "mx_ab failed"; tail -30 gpurun_out/mx_ab.log; return 1; }
  grep '^{' gpurun_out/mx_ab.log
}

case "${1:?study: counters|models|grpc|qps|trace|embed|gemm}" in
  counters|models|grpc|qps|trace|embed|gemm) "$1" ;;
  *) echo "unknown study $1"; exit 2 ;;
esac

#!/bin/bash
# Round-4 GPU steps on one MI355X; each step under its own time limit, the script stops at the first failure.
#   MODELS="deepfm" COUNTERS="deepfm dlrm dcn_v2" TESTS="tests/test_kernels_gpu.py" bash scripts/gpu_r4.sh
# Counter passes (rocprofv3 --pmc, one run each, kernel trace only - never with a sys/runtime trace):
#   SQ occupancy + MFMA + LDS | FETCH_SIZE | WRITE_SIZE + L2 hit | wait / issue-stall / active shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r4.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r4.log; exit 1; }
  tail -3 gpurun_out/pytest_r4.log
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/smoke.log
fi
if [ -n "${STUDY:-}" ]; then
  timeout -k 10 ${STUDY_TIMEOUT:-300} python -u -m $STUDY ${STUDY_ARGS:-} > gpurun_out/study.log 2>&1 \
    || { echo "study failed"; tail -30 gpurun_out/study.log; exit 1; }
  cat gpurun_out/study.log
fi
for m in ${MODELS:-}; do
  timeout -k 10 400 python -u bench.py --model $m --steps ${STEPS:-200} --warmup 20 ${BENCH_ARGS:-} \
    > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -40 gpurun_out/bench_$m.log; exit 1; }
  grep '^{"metric' gpurun_out/bench_$m.log | cut -c1-1500
done
if [ -n "${BENCHES:-}" ]; then
  # ';'-separated bench.py argument sets, e.g. BENCHES="--model dlrm;--model dlrm --shard-tables"
  IFS=';' read -ra SETS <<< "$BENCHES"
  i=0
  for args in "${SETS[@]}"; do
    i=$((i+1))
    # leading VAR=value words are environment settings for this set (e.g. "DTFS_RESOLVE_LANE=1 --model deepfm")
    envs=(); rest=()
    for w in $args; do
      if [ ${#rest[@]} -eq 0 ] && [[ $w =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$w"); else rest+=("$w"); fi
    done
    timeout -k 10 500 env "${envs[@]}" python -u bench.py "${rest[@]}" --steps ${STEPS:-200} --warmup 20 > gpurun_out/bench_set$i.log 2>&1 \
      || { echo "bench [$args] failed"; tail -40 gpurun_out/bench_set$i.log; exit 1; }
    echo "[$args]"; grep '^{"metric' gpurun_out/bench_set$i.log | cut -c1-2500
  done
fi
if [ "${REF:-0}" = "1" ]; then
  # the reference workload in process, then over TCP from a separate process of native h2c clients
  timeout -k 10 300 python -u bench.py --reference-workload > gpurun_out/bench_ref.log 2>&1 \
    || { echo "reference workload failed"; tail -30 gpurun_out/bench_ref.log; exit 1; }
  grep -E '^Average|^\{' gpurun_out/bench_ref.log | cut -c1-1200
  timeout -k 10 400 python -u bench.py --reference-workload --over-grpc --grpc-threads ${GRPC_THREADS:-4} \
    > gpurun_out/bench_ref_grpc.log 2>&1 || { echo "reference workload over gRPC failed"; tail -30 gpurun_out/bench_ref_grpc.log; exit 1; }
  grep -E '^Average|^\{' gpurun_out/bench_ref_grpc.log | cut -c1-1500
fi
if [ -n "${COUNTERS:-}" ]; then
  OUT=gpurun_out/ctr4
  rm -rf $OUT && mkdir -p $OUT
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  P2="FETCH_SIZE GRBM_GUI_ACTIVE"
  P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  P4="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
  for model in $COUNTERS; do
    rows=16384; [ $model = dcn_v2 ] && rows=8192
    i=0
    for pass in "$P1" "$P2" "$P3" "$P4"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/${model}_p$i -o run \
        -- python3 -m tools.studies.kernel_drive --model $model --rows $rows --iters 10 \
        > $OUT/${model}_p$i.log 2>&1 || { echo "pass $i of $model failed"; tail -5 $OUT/${model}_p$i.log; exit 1; }
    done
    python -m tools.counters_summary $OUT --only ${model}_ \
      --title "$model serving-shape forward ($rows rows), 1 MI355X (rocprofv3 --pmc, 4 passes)" > $OUT/summary_$model.md
    cat $OUT/summary_$model.md
    rm -rf $OUT/${model}_p*  # raw CSVs: tens of MB each (gpurun copies back <= 64 MiB)
  done
fi
if [ -n "${PROF_MODELS:-}" ]; then
  for pm in $PROF_MODELS; do
    tag=$pm${PROF_TAG:+_$PROF_TAG}
    rm -rf gpurun_out/prof_$tag
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_$tag -o run --output-format rocpd \
      -- python3 bench.py --model $pm --steps 100 --warmup 10 --qps 0 ${BENCH_ARGS:-} > gpurun_out/prof_$tag.log 2>&1 \
      || { echo "prof $pm failed"; tail -30 gpurun_out/prof_$tag.log; exit 1; }
    db=$(find gpurun_out/prof_$tag -name '*.db' | head -1)
    case $pm in deepfm|wdl|dcn) sk="gemm_gather --min-us 60";; dlrm) sk="bottom_mlp3 --min-us 14";; *) sk="embed_pipe --min-us 30";; esac
    python -m tools.prof_summary "$db" --steps ${PROF_STEPS:-110} --step-kernel $sk \
      --title "bench.py live path ($pm ${BENCH_ARGS:-} ${PROF_TAG:-}), 1 MI355X" > gpurun_out/prof_summary_$tag.md \
      && head -30 gpurun_out/prof_summary_$tag.md
    rm -f "$db"  # the summary is what travels back (the rocpd database is tens of MB)
  done
fi
echo "gpu_r4 done"

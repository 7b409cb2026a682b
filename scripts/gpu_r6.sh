#!/bin/bash
# Round-6 GPU steps on one MI355X; each step under its own time limit, the script stops at the first failure.
#   TESTS="tests" SMOKE=1 BENCHES="--model deepfm;--model dlrm" PROFS="deepfm|--model deepfm;ff|--model deepfm --force-fanout" \
#     COUNTERS="deepfm dcn_v2" STUDY=tools.studies.microbench STUDY_ARGS=--tail bash scripts/gpu_r6.sh
# BENCHES / PROFS: ';'-separated bench.py argument sets (leading VAR=value words are environment settings);
# PROFS entries are tag|args: a kernel + copy trace (rocprofv3 --kernel-trace --memory-copy-trace --stats,
# never with counters) summarised by tools/prof_summary.py into gpurun_out/prof_summary_<tag>.md.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
split_env() {  # "A=1 B=2 --x y" -> envs=(A=1 B=2) rest=(--x y)
  envs=(); rest=()
  for w in $1; do
    if [ ${#rest[@]} -eq 0 ] && [[ $w =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$w"); else rest+=("$w"); fi
  done
}
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_r6.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r6.log; exit 1; }
  tail -3 gpurun_out/pytest_r6.log
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
if [ -n "${COUNTERS:-}" ]; then
  # counter passes (rocprofv3 --pmc, one run each, kernel trace only - never with a sys/runtime trace)
  OUT=gpurun_out/ctr6
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
if [ -n "${BENCHES:-}" ]; then
  IFS=';' read -ra SETS <<< "$BENCHES"
  i=0
  for args in "${SETS[@]}"; do
    i=$((i+1))
    split_env "$args"
    timeout -k 10 ${BENCH_TIMEOUT:-400} env "${envs[@]}" python -u bench.py "${rest[@]}" --steps ${STEPS:-200} --warmup 20 \
      > gpurun_out/bench_set$i.log 2>&1 || { echo "bench [$args] failed"; tail -40 gpurun_out/bench_set$i.log; exit 1; }
    echo "[$args]"; grep '^{"metric' gpurun_out/bench_set$i.log | cut -c1-3000
  done
fi
if [ -n "${PROFS:-}" ]; then
  IFS=';' read -ra SETS <<< "$PROFS"
  for spec in "${SETS[@]}"; do
    tag=${spec%%|*}; args=${spec#*|}
    split_env "$args"
    rm -rf gpurun_out/prof_$tag
    timeout -k 10 300 env "${envs[@]}" rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_$tag -o run \
      --output-format rocpd -- python3 bench.py "${rest[@]}" --steps 100 --warmup 10 --qps 0 --qps-sweep= \
      > gpurun_out/prof_$tag.log 2>&1 || { echo "prof $tag failed"; tail -30 gpurun_out/prof_$tag.log; exit 1; }
    db=$(find gpurun_out/prof_$tag -name '*.db' | head -1)
    case "$args" in *dlrm*) sk="bottom_mlp3 --min-us 14";; *dcn_v2*) sk="embed_pipe --min-us 30";; *"model dcn "*|*"model dcn") sk="gemm_gather --min-us 60";; *) sk="gather_mlp --min-us 60";; esac
    python -m tools.prof_summary "$db" --steps ${PROF_STEPS:-110} --step-kernel $sk \
      --title "bench.py live path ($args), 1 MI355X" > gpurun_out/prof_summary_$tag.md \
      && head -40 gpurun_out/prof_summary_$tag.md
    rm -f "$db"  # the summary travels back (the rocpd database is tens of MB)
  done
fi
echo "gpu_r6 done"

#!/bin/bash
# Gather-GEMM (K1 fused into K4) on one MI355X: its GPU tests, the kernel
# study, then a DeepFM bench + kernel profile. Each step under its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "embed_gemm or gather_gemm or test_head or linear_head or models_gpu_vs_cpu or forward_arena or dense_pad" \
  > gpurun_out/gg_tests.log 2>&1 || { echo "gather-GEMM tests failed"; tail -40 gpurun_out/gg_tests.log; exit 1; }
tail -3 gpurun_out/gg_tests.log
timeout -k 10 200 python -u -m tools.studies.microbench --gather-gemm > gpurun_out/gg_study.log 2>&1 \
  || { echo "study failed"; tail -20 gpurun_out/gg_study.log; exit 1; }
grep '^{' gpurun_out/gg_study.log
if [ "${LIVE:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_live_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/gg_live.log 2>&1 || { echo "live tests failed"; tail -40 gpurun_out/gg_live.log; exit 1; }
  tail -3 gpurun_out/gg_live.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  for m in ${MODELS:-deepfm}; do
    timeout -k 10 300 python -u bench.py --model $m --steps 200 --warmup 20 --json-extra > gpurun_out/gg_bench_$m.log 2>&1 \
      || { echo "bench $m failed"; tail -30 gpurun_out/gg_bench_$m.log; exit 1; }
    grep '^{"metric' gpurun_out/gg_bench_$m.log | cut -c1-300
  done
fi
if [ "${PROFILE:-1}" = "1" ]; then
  rm -rf gpurun_out/prof_gg
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_gg -o run --output-format rocpd \
    -- python3 bench.py --model ${PROF_MODEL:-deepfm} --steps 100 --warmup 10 --qps 0 > gpurun_out/prof_gg.log 2>&1 \
    || { echo "prof failed"; tail -30 gpurun_out/prof_gg.log; exit 1; }
  db=$(find gpurun_out/prof_gg -name '*.db' | head -1)
  python -m tools.prof_summary "$db" --from-kernel gemm_head --title "bench.py live path (${PROF_MODEL:-deepfm}, gather-GEMM), 1 MI355X" \
    > gpurun_out/prof_summary_gg.md && head -24 gpurun_out/prof_summary_gg.md
fi

#!/bin/bash
# Host + device timeline of the live bench: roctx ranges of the live server
# (DTFS_TRACE=1: live_build / live_launch / live_wait / live_encode) with the
# kernel and memory-copy traces, for lining up launches with H2D and kernels.
set -o pipefail
export TMPDIR=/tmp DTFS_TRACE=1
rm -rf gpurun_out/tl && mkdir -p gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format rocpd -d gpurun_out/tl -o run \
  -- python3 bench.py --steps 60 --warmup 10 --qps 0 ${ARGS:-} > gpurun_out/tl/bench.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/tl/bench.log; exit 1; }
grep '^{"metric' gpurun_out/tl/bench.log | cut -c1-300

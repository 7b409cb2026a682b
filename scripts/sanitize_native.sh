#!/usr/bin/env bash
# ASan + UBSan run of the host runtime (wire codec, request arena, batcher,
# thread pool) under the CPU test suites. Host code only:
# GPU sanitizers are not available on the MI355X pool.
set -euo pipefail
cd "$(dirname "$0")/.."
python -m distributed_tf_serving_amd._build --sanitize
ASAN_LIB=$(g++ -print-file-name=libasan.so)
UBSAN_LIB=$(g++ -print-file-name=libubsan.so)
status=0
LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 DTFS_NO_AUTOBUILD=1 \
  python -m pytest tests/test_wire.py tests/test_runtime_cpu.py tests/test_serving_e2e.py tests/test_faults.py \
  -q -m "not gpu" -p no:cacheprovider "$@" || status=$?
# restore the optimised build
python -m distributed_tf_serving_amd._build --native-only --force >/dev/null
exit $status

#!/usr/bin/env bash
# Host sanitizer runs of the native runtime (wire codec, request arena, batcher,
# thread pool, live server, step control, load generator) under the CPU test
# suites. Host code only: GPU sanitizers are not available on
# the MI355X pool.
#   bash scripts/sanitize_native.sh            # ASan + UBSan, then TSan
#   SAN=address bash scripts/sanitize_native.sh tests/test_bench_cpu.py
#   SAN=thread  bash scripts/sanitize_native.sh   # TSan + ASan on tools/native/live_stress.cpp
set -uo pipefail
cd "$(dirname "$0")/.."
SAN=${SAN:-both}
if [ $# -gt 0 ]; then SUITES="$*"; else
  SUITES="tests/test_wire.py tests/test_runtime_cpu.py tests/test_serving_e2e.py tests/test_faults.py \
tests/test_live_server.py tests/test_arena_cpu.py tests/test_step_control.py tests/test_bench_cpu.py \
tests/test_cluster_server.py tests/test_shared_scatter.py tests/test_native_front.py"
fi
status=0
if [ "$SAN" = address ] || [ "$SAN" = both ]; then
  SO=$(python -m distributed_tf_serving_amd._build --sanitize address | tail -1) || exit 1
  ASAN_LIB=$(g++ -print-file-name=libasan.so)
  UBSAN_LIB=$(g++ -print-file-name=libubsan.so)
  # detect_stack_use_after_return: run_load's completion-callback race (round 3) was exactly that
  LD_PRELOAD="$ASAN_LIB $UBSAN_LIB" \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:detect_stack_use_after_return=1 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 DTFS_NO_AUTOBUILD=1 DTFS_NATIVE_SO="$SO" \
    python -m pytest $SUITES -q -m "not gpu" -p no:cacheprovider || status=$?
  echo "asan+ubsan: exit $status"
fi
if [ "$SAN" = thread ] || [ "$SAN" = both ]; then
  # ThreadSanitizer on a C++-only driver of the same objects (tools/native/live_stress.cpp: live
  # server + load generator + thread pool + two ranks on one step control). Under the Python suites
  # TSan reports noise: the interpreter / torch are uninstrumented and gcc 11's libtsan misses
  # pthread_cond_clockwait (std::condition_variable::wait_for), so ROCm's clang TSan runtime is used.
  CLANG=/opt/rocm/lib/llvm/bin/clang++
  SRCS="tools/native/live_stress.cpp csrc/runtime/live_server.cpp csrc/runtime/loadgen.cpp csrc/runtime/step_control.cpp \
csrc/runtime/arena.cpp csrc/runtime/narrow.cpp csrc/runtime/batcher.cpp csrc/runtime/thread_pool.cpp csrc/runtime/trace.cpp \
csrc/runtime/shared_scatter.cpp csrc/runtime/numa.cpp csrc/wire/tensor_codec.cpp"
  mkdir -p build/stress
  t=0
  $CLANG -O1 -g -std=c++17 -fsanitize=thread -fno-omit-frame-pointer -Icsrc $SRCS -o build/stress/live_stress_tsan \
    -lpthread -ldl -lrt && TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1" timeout 600 build/stress/live_stress_tsan \
    || t=$?
  echo "tsan (live_stress): exit $t"
  [ $t = 0 ] || status=$t
  a=0
  $CLANG -O1 -g -std=c++17 -fsanitize=address,undefined -fno-omit-frame-pointer -Icsrc $SRCS \
    -o build/stress/live_stress_asan -lpthread -ldl -lrt && \
    ASAN_OPTIONS=detect_stack_use_after_return=1:abort_on_error=1 timeout 600 build/stress/live_stress_asan || a=$?
  echo "asan (live_stress): exit $a"
  [ $a = 0 ] || status=$a
fi
# the instrumented _native was built under build/ (DTFS_NATIVE_SO): the in-tree .so is untouched
exit $status

// Native load generator for a LiveServer (in-process clients).
//
// Drives LiveServer::submit() - the same entry point the gRPC front door and
// the in-process PredictionService use - from C++ client threads, so a
// benchmark measures the served path (admission, batching, one copy into the
// pinned arena, parse, launch, encode, completion) and not a Python client.
// Reference counterpart: the closed-loop driver of DCNClient.main (6 threads
// x 1000 back-to-back requests, reference DCNClient.java:205-241); the
// open-loop fixed-QPS mode is what BASELINE.json's "p50 request latency at
// fixed QPS" needs (the reference has no such mode).
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "live_server.h"

namespace dtfs {
namespace runtime {

struct LoadSpec {
  int64_t warmup = 0;       // completions before the timed window opens
  int64_t count = 0;        // completions inside the timed window
  int64_t tail = -1;        // closed loop: extra requests after the window (keeps it steady; -1 = concurrency)
  int concurrency = 64;     // closed loop: requests outstanding at all times
  double qps = 0;           // > 0: open loop, requests sent on a fixed schedule
  bool poisson = false;     // open loop: exponential inter-arrival times instead of uniform
  int threads = 4;          // submitting threads (each copies its requests into the arena)
  int64_t timeout_us = 0;   // per-request deadline (0 = none)
  uint64_t seed = 1;
  int64_t debug_done_delay_us = 0;  // test hook: the last request's completion callback sleeps this long
                                    // after its completion is counted (run_load must still wait for it)
};

// Stages of one request's latency (us), in order: sched_lag (open loop: the
// submitting thread picked it up late), admit (until admitted into an arena:
// a full server blocks here), batch (admitted -> its step launched: batching
// wait + build + launch), step (launched -> the completer saw it done: the GPU
// step and the steps ahead of it), encode (the batch's responses up to this
// one), deliver (encoded -> the client's callback ran).
constexpr int kStages = 6;
using Stages = std::array<float, kStages>;

struct LoadResult {
  std::vector<double> latency_us;  // timed requests (closed loop: completion order; open loop: by schedule)
  std::vector<Stages> stages_us;   // the same requests' stages, same order (OK replies only: else zeros)
  int64_t submitted = 0, ok = 0, errors = 0;
  double window_us = 0;            // timed window: first to last timed completion boundary
  double wall_us = 0;
  std::string first_error;
  int first_error_code = 0;
};

LoadResult run_load(LiveServer& srv, const std::vector<std::string>& requests, const LoadSpec& spec);

}  // namespace runtime
}  // namespace dtfs

// Native serving loop: the per-rank hot loop of the shard backend, in C++.
//
// One step = a batch of client PredictRequests sitting in a pinned request
// arena (serving/arena.py) ->
//   parse   : protobuf framing -> arena descriptors (csrc/runtime/arena.cpp)
//   launch  : SDMA H2D of the arena + the step graph (GPU unpack -> forward ->
//             scores written into pinned host memory), or the fan-out step
//             (StepRunner.launch_fanout: collectives over RCCL)
//   finish  : wait for the step's completion event
//   encode  : one PredictResponse per request (prediction_node float_val)
// on three threads (parser, launcher = the caller, encoder) with `depth` steps
// in flight on the GPU and S >= depth + 1 slots of device/host buffers.
//
// This replaces, per rank, what the reference delegates to a TF-Serving host
// (reference DCNClient.java:111-112 Predict RPC; README.md:5 server batching)
// and keeps Python entirely out of the steady-state loop.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "arena.h"
#include "step_runner.h"

namespace dtfs {
namespace runtime {

struct LoopSlot {
  void* h2d_dst = nullptr;           // device arena of the slot (local launch)
  int64_t h2d_cap = 0;               // its size in bytes
  hipGraphExec_t graph = nullptr;    // local: unpack + forward + scores -> h_out
  const KernelSequence* seq = nullptr;  // local, preferred: the same step as direct launches
  bool fanout = false;
  FanoutStep fan;                    // fan-out: everything but h2d_src / h2d_bytes
  bool program = false;
  StepProgram prog;                  // programmed step (embedding-parallel models)
  const float* h_out = nullptr;      // pinned scores of the slot
  int64_t h_out_len = 0;
};

struct LoopConfig {
  int depth = 3;
  int64_t fields = 43;
  int64_t max_rows = 0;
  int64_t varint_chunks = 0;  // > 0: packed varint ids are decoded on the GPU (arena.h)
  std::string ids_key = "feat_ids", wts_key = "feat_wts";
  std::string model_name = "DCN", signature_name = "serving_default", output_key = "prediction_node";
  int64_t version = -1;  // < 0: unset
};

struct LoopStats {
  std::vector<double> latency_us;  // per step: parse start -> scores on the host
  std::vector<double> score_sum;   // per step: sum of the scores the encoder read (record only)
  int64_t steps = 0, requests = 0, rows = 0, errors = 0, response_bytes = 0;
  double parse_us = 0, launch_us = 0, wait_us = 0, encode_us = 0, wall_us = 0;
};

class ServingLoop {
 public:
  ServingLoop(StepRunner* runner, LoopConfig cfg, std::vector<LoopSlot> slots);
  // Register one pre-received request batch (arena + request spans). Inputs are
  // used round-robin; an arena is re-parsed only after its previous step ended.
  void add_input(uint8_t* arena, int64_t capacity, std::vector<Span> spans);
  LoopStats run(int64_t n_steps, bool record = true);
  int slots() const { return int(slots_.size()); }

 private:
  struct Input {
    uint8_t* arena;
    int64_t capacity;
    std::vector<Span> spans;
  };
  StepRunner* runner_;
  LoopConfig cfg_;
  std::vector<LoopSlot> slots_;
  std::vector<Input> inputs_;
};

}  // namespace runtime
}  // namespace dtfs

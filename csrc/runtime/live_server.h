// Live serving core: concurrent PredictRequests in, PredictResponses out,
// with server-side dynamic batching straight into pinned request arenas.
//
// This is the per-rank TF-Serving ModelServer hot path (reference
// DCNClient.java:111-112 is the client side of it; README.md:5,9 the batching
// it relies on), with no Python and no per-request allocation on the way:
//
//   submit() (any thread: gRPC workers, in-process clients, the native load
//            generator)   framing parse -> admission -> reserve a span in the
//            OPEN arena -> memcpy the request bytes into pinned memory
//   launcher thread       closes a batch (max rows / batch timeout / device
//            idle), parses framing into arena descriptors (arena.cpp), picks the
//            smallest bucket >= rows, waits for a free slot, launches the step
//            (StepBackend: SDMA H2D + kernels, or the fan-out step)
//   completer thread      waits for the step (bounded: a stuck step or an RCCL
//            error fails the in-flight requests UNAVAILABLE and marks the server
//            broken instead of hanging), encodes one PredictResponse per
//            request, runs its completion, recycles slot + arena
//
// Request bytes are copied exactly once, by the thread that received them,
// into memory the DMA engine reads directly. The device work is behind
// StepBackend so the same core serves a GPU (csrc/bindings_hip.cpp: StepRunner
// + captured step kernels) and a CPU backend (csrc/bindings_native.cpp:
// a Python forward; Wide&Deep-tiny BASELINE config 1, and the CPU tests).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "arena.h"
#include "step_control.h"

namespace dtfs {
namespace runtime {

// gRPC status codes used in replies (grpc/status.h numbering).
enum StatusCode : int {
  kOk = 0,
  kInvalidArgument = 3,
  kDeadlineExceeded = 4,
  kNotFound = 5,
  kResourceExhausted = 8,
  kInternal = 13,
  kUnavailable = 14,
  // not a gRPC code: the request has more rows than one batch holds; the
  // caller may split it and resubmit the parts (serving/batching.py does)
  kOversize = 1000,
  // not a gRPC code: the request asks for an output the fast path does not
  // produce (LiveConfig::caller_outputs, e.g. the ranked outputs); the
  // caller's general path serves it (serving/service.py)
  kCallerPath = 1001,
};

struct Reply {
  int code = kOk;
  std::string message;
  std::string response;  // serialized PredictResponse when code == kOk
  // steady-clock microseconds (now_us()) of the request's life in the server,
  // 0 when it never got there: admitted into an arena, its step launched, the
  // step seen done by the completer, its response encoded. The load generator
  // splits each latency into these stages (where a tail request waited).
  int64_t t_arrive = 0, t_launch = 0, t_done = 0, t_encoded = 0;
};
using Completion = std::function<void(Reply&&)>;

// The device side of a live server: `slots()` step slots, each able to run one
// batch of a given bucket (padded row count) from a parsed host arena.
class StepBackend {
 public:
  virtual ~StepBackend() = default;
  virtual int slots() const = 0;
  virtual const std::vector<int64_t>& buckets() const = 0;  // ascending
  // Enqueue one step of bucket index `b` on `slot` reading `arena` (pinned;
  // `batch` is its parse). Must not block on the device.
  virtual void launch(int slot, int b, const uint8_t* arena, const ArenaBatch& batch) = 0;
  // Wait for the slot's last step. false: not done within timeout_us (or an
  // asynchronous communicator error, described in *err).
  virtual bool wait(int slot, int64_t timeout_us, std::string* err) = 0;
  virtual const float* scores(int slot, int b) const = 0;
  virtual int64_t scores_len(int slot, int b) const = 0;
  // Called once when the server gives up on the device (stuck step / error):
  // abort communicators so peers stop waiting on this rank.
  virtual void abort() {}
};

struct LiveConfig {
  int64_t fields = 43;
  std::string ids_key = "feat_ids", wts_key = "feat_wts";
  std::string model_name = "DCN", signature_name = "serving_default", output_key = "prediction_node";
  int64_t version = -1;            // < 0: unversioned
  int64_t max_batch_rows = 0;      // 0: the largest bucket
  int64_t batch_timeout_us = 200;  // oldest queued request waits at most this long
  int depth = 3;                   // steps in flight (<= slots)
  int64_t varint_chunks = 0;       // GPU varint decode capacity (arena.h)
  int64_t max_pending = 1 << 16;   // admitted, unfinished requests; beyond: RESOURCE_EXHAUSTED
  bool eager_when_idle = true;     // no step in flight: launch what is queued right away
  int64_t step_timeout_us = 10'000'000;  // a GPU step taking longer = the device / a peer is gone
  // Cluster mode (a StepControl is given: collectives inside the step): steps
  // are agreed with the other ranks (step_control.h). A peer whose heartbeat
  // is older than peer_timeout_us breaks the cluster; heartbeat_us is the
  // watcher's period.
  int64_t peer_timeout_us = 5'000'000;
  // liveness_only: the StepControl only carries heartbeats and the broken flag
  // (ranks whose steps have no collectives but read each other's memory: the
  // sharded DLRM's peer exchange maps every owner's tables by IPC). Steps are
  // not agreed; a silent peer still breaks this server (UNAVAILABLE).
  bool liveness_only = false;
  int64_t heartbeat_us = 20'000;
  // Launch nothing until resume() (requests are admitted and queue): a server
  // whose step issues torch.distributed collectives from the launcher thread
  // must not launch before every rank has finished its start-up collectives.
  bool start_paused = false;
  // > 0: requests with raw tensor_content int64 ids + fp32 weights are
  // narrowed by the submitting thread while it copies them (runtime/narrow.h):
  // ids -> table rows (id mod narrow_modulo: the model's table size) as 3-byte
  // rows when the table has <= 2^24 rows, else int32; weights stay fp32 (7 or
  // 8 bytes per feature instead of 12); other encodings travel raw.
  int64_t narrow_modulo = 0;
  // > 0 (narrowed requests only): keep just the first narrow_wts_cols weights
  // of each row - the model reads no others (one-hot DLRM: the dense
  // features; its sparse fields' weights are unused). Fewer H2D bytes; the
  // arena header tells the GPU readers, which see 0 for the dropped columns.
  int64_t narrow_wts_cols = 0;
  // output keys the signature has besides output_key that only the caller's
  // general path produces: a request naming one in output_filter gets
  // kCallerPath instead of INVALID_ARGUMENT
  std::vector<std::string> caller_outputs;
};

struct LiveStats {
  int64_t submitted = 0, rejected = 0, completed = 0, failed = 0, expired = 0;
  int64_t steps = 0, rows = 0, padded_rows = 0, empty_steps = 0;
  int64_t full_steps = 0, timeout_steps = 0, eager_steps = 0, blocked_submits = 0, narrowed = 0;
  // narrowed requests whose weights travelled as bf16 (all exact) / not at all (all 1.0)
  int64_t narrowed_wts_bf16 = 0, narrowed_wts_implicit = 0;
  // cluster mode: steps this rank proposed / joined with a batch of its own /
  // joined with nothing queued (empty_steps counts those too)
  int64_t proposed_steps = 0, joined_steps = 0;
  double copy_us = 0, build_us = 0, launch_us = 0, wait_us = 0, encode_us = 0;
  bool broken = false;
  std::string error;
};

class LiveServer {
 public:
  // bytes per host-narrowed id: 3 when every row fits 24 bits, else 4
  int64_t narrow_id_bytes() const {
    return cfg_.narrow_modulo > 0 && cfg_.narrow_modulo <= (int64_t(1) << 24) ? 3 : 4;
  }
  // arenas: pinned host buffers of ArenaLayout capacity (>= 2 + depth of them).
  // ctl: cluster mode (every step agreed with the other ranks), or null.
  LiveServer(StepBackend* backend, LiveConfig cfg, std::vector<std::pair<uint8_t*, int64_t>> arenas,
             StepControl* ctl = nullptr);
  ~LiveServer();
  LiveServer(const LiveServer&) = delete;
  LiveServer& operator=(const LiveServer&) = delete;

  // Admit one serialized PredictRequest; its bytes are copied before this
  // returns. `done` runs exactly once: on the completer thread, or on the
  // caller's thread for an immediate rejection. deadline_us: absolute
  // steady-clock microseconds (now_us()), 0 = none; a submitter that finds
  // every arena busy waits for one until then.
  void submit(const uint8_t* data, size_t n, int64_t deadline_us, Completion done);
  // Never blocks: false (done untouched, nothing admitted) when every arena is
  // queued or in flight and submit() would wait for one; otherwise as submit().
  // Event-loop callers hand a false over to a thread that may block.
  bool try_submit(const uint8_t* data, size_t n, int64_t deadline_us, Completion& done);
  // Blocking convenience wrapper.
  Reply predict(const uint8_t* data, size_t n, int64_t deadline_us);

  // Stop admitting; launch what is queued, finish every step in flight.
  void close();
  // Start launching (see LiveConfig::start_paused).
  void resume();
  LiveStats stats() const;
  bool broken() const { return broken_.load(); }
  int64_t max_rows() const { return max_rows_; }
  const LiveConfig& config() const { return cfg_; }

 private:
  bool admit(const uint8_t* data, size_t n, int64_t deadline_us, Completion& done, bool wait);
  struct Pending {
    int64_t off, len, rows, deadline_us, t_arrive;
    Completion done;
    bool narrow = false;
    int64_t ids_off = 0, wts_off = 0;  // narrow: payload offsets of the 3-byte / int32 rows and the weights
    int wkind = 0;                     // narrow: WtsKind of the weights (runtime/narrow.h)
  };
  struct Arena {
    uint8_t* base = nullptr;
    int64_t capacity = 0;
    int64_t used = 0, rows = 0, need = 0, t_first = 0;
    int writers = 0;
    std::vector<Pending> pend;
  };
  struct InFlight {
    int arena, slot, bucket;
    ArenaBatch batch;
    std::vector<Pending> pend;  // same order as the spans handed to arena_build
    int64_t t_launch;
  };

  void launcher_loop();
  void completer_loop();
  void watcher_loop();  // cluster mode: heartbeats, peer liveness, wakes an idle launcher
  int bucket_for(int64_t rows) const;
  int64_t need_of(int64_t len, int64_t rows) const;
  void fail_all(std::vector<Pending>& ps, int code, const std::string& msg);
  void go_broken(const std::string& why);  // call WITHOUT mu_ held
  void release(int arena, int slot);

  StepBackend* backend_;
  LiveConfig cfg_;
  StepControl* ctl_ = nullptr;    // heartbeats + the cluster's broken flag (watcher thread)
  StepControl* agree_ = nullptr;  // ctl_ unless liveness_only: every step agreed with the other ranks
  int64_t max_rows_ = 0;
  int64_t arena_budget_ = 0;  // payload bytes a batch may plan for (see need_of)

  mutable std::mutex mu_;
  std::condition_variable cv_launch_;  // launcher: new work / slot freed / writers done
  std::condition_variable cv_space_;   // submitters: an arena became free
  std::condition_variable cv_done_;    // completer: a step was launched
  std::vector<Arena> arenas_;
  std::deque<int> free_, sealed_;
  int open_ = -1;
  std::vector<char> slot_busy_;
  int next_slot_ = 0;
  int inflight_ = 0;
  int64_t pending_ = 0;
  int64_t steps_launched_ = 0;
  bool closing_posted_ = false, watcher_stop_ = false;
  std::atomic<bool> launcher_idle_{false};
  std::deque<InFlight> q_done_;
  bool closing_ = false, launcher_exited_ = false, paused_ = false;
  std::atomic<bool> broken_{false};
  std::string error_;
  LiveStats st_;

  std::thread launcher_, completer_, watcher_;
};

}  // namespace runtime
}  // namespace dtfs

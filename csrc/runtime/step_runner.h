// Native per-GPU step launcher: the hot loop of the shard backend without
// Python in it.
//
// One serving step on a GPU is
//     H2D(packed request rows)  ->  hipGraphLaunch(forward + D2H of scores)
// with the H2D on its own stream so the SDMA engine moves step k+1's rows while
// step k's kernels run. StepRunner owns the streams and events, takes the
// instantiated graph of each (bucket, slot) by its raw hipGraphExec_t handle
// (captured once from PyTorch), and enqueues a whole step in ~4 HIP API calls.
// wait() blocks in hipEventSynchronize with the GIL released by the binding.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../comm/rccl_comm.h"
#include "kernel_seq.h"
#include "shared_scatter.h"  // ShareCopy

namespace dtfs {
namespace runtime {

// One fan-out step (world > 1), all pointers device unless noted:
//   copy stream : H2D h2d_src (pinned host) -> h2d_dst
//   ingress     : [ingress graph, e.g. GPU unpack of the request arena]
//                 -> collective-in (all-to-all / scatter of packed rows)
//   compute     : forward graph (recv rows -> scores)
//   egress      : collective-out (all-to-all / gather of scores) -> D2H
// Ingress and egress have their own streams and communicators, so step k+1's
// row exchange and step k-1's score exchange overlap step k's forward.
struct FanoutStep {
  void* h2d_dst = nullptr;
  const void* h2d_src = nullptr;
  int64_t h2d_bytes = 0;
  hipGraphExec_t ingress = nullptr;
  comm::RcclComm* cin = nullptr;
  int mode = 0;  // 0 = all-to-all, 1 = scatter from / gather to rank 0
  const void* send = nullptr;
  void* recv = nullptr;
  size_t in_bytes = 0;   // per peer
  hipGraphExec_t forward = nullptr;
  comm::RcclComm* cout = nullptr;
  const void* scores = nullptr;
  void* back = nullptr;
  size_t out_bytes = 0;  // per peer
  void* h_out = nullptr;  // pinned host
  size_t d2h_bytes = 0;
  // optional: replay these instead of launching the graphs (same kernels)
  const KernelSequence* ingress_seq = nullptr;
  const KernelSequence* forward_seq = nullptr;
  // optional: the forward's front half (the gather-GEMM's resolve pass) on the
  // ingress lane right after the row exchange, so step k+1's resolve runs
  // beside step k's forward (the local two-lane program's split, fan-out form)
  hipGraphExec_t resolve = nullptr;
  const KernelSequence* resolve_seq = nullptr;
  // no request of the step carries packed varint ids: the ingress sequence
  // leaves out the arena varint-decode kernel
  bool skip_varint = false;
};

// A step as a short program over two device lanes - the compute stream and
// an auxiliary stream - for models whose forward interleaves collectives with
// kernels (embedding model parallelism, SURVEY §2.5 C3: ids all-to-all ->
// owner-side gather -> embeddings all-to-all on the aux lane while the bottom
// MLP runs on the compute lane). Ops run in list order on their lane; lanes
// meet only through kRecord / kWait on per-slot events. The H2D lands before
// the lane named by h2d_lane starts; the step is done when the compute lane
// is, so every aux-lane op must be joined into the compute lane (validated).
// All ranks enqueue the same collectives in the same order on the aux lane
// with one communicator, so the exchange cannot cross-match between steps.
struct ProgOp {
  enum Kind : int {
    kKernels = 0,        // seq (direct launches) or graph
    kAllToAll = 1,       // comm: send -> recv, `bytes` per peer
    kAllGather = 2,      // comm: send (`bytes`) -> recv (W x bytes)
    kReduceScatter = 3,  // comm: bf16 sum, send (W x elems) -> recv (`bytes` = elems)
    kRecord = 4,         // record per-slot event `event` on the lane
    kWait = 5,           // lane waits for per-slot event `event`
    kWaitPrev = 6,       // lane waits for event `event` of the PREVIOUS programmed step (any slot;
                         // no-op for the first): cross-step overlap, e.g. step k+1's gather
                         // starts when step k's first GEMM is done, so it shares the CUs with
                         // step k's smaller GEMMs instead of delaying the big one
  };
  int kind = kKernels;
  int lane = 0;  // 0 compute, 1 aux
  int event = 0;
  const KernelSequence* seq = nullptr;
  hipGraphExec_t graph = nullptr;
  comm::RcclComm* comm = nullptr;
  const void* send = nullptr;
  void* recv = nullptr;
  size_t bytes = 0;
};
constexpr int kProgEvents = 8;

struct StepProgram {
  void* h2d_dst = nullptr;
  int h2d_lane = 1;
  std::vector<ProgOp> ops;
  // throws std::invalid_argument when an event index is out of range, an
  // event is waited before it is recorded, or aux-lane work is never joined
  // into the compute lane
  void validate() const;
};

// What one (bucket, slot) of a live server launches: a local step (direct
// launches of the captured step, or its graph), a fan-out step, or a
// programmed step; plus the pinned host scores it produces.
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

class StepRunner {
 public:
  StepRunner(int device, int slots);
  ~StepRunner();
  StepRunner(const StepRunner&) = delete;
  StepRunner& operator=(const StepRunner&) = delete;

  // Enqueue one step on `slot`: copy nbytes host->device (pinned src), then
  // launch graph_exec on the compute stream once the copy has landed. The H2D
  // waits only for the previous step of the same slot to have consumed dst.
  void launch(int slot, void* dst, const void* src, int64_t nbytes, hipGraphExec_t graph);
  // Same, replaying the step as direct kernel launches (no graph-launch gap).
  void launch_seq(int slot, void* dst, const void* src, int64_t nbytes, const KernelSequence* seq,
                  bool skip_varint = false);
  // Same, with the H2D as several copies into dst (a rank's share of a
  // shared-scatter batch, runtime/shared_scatter.h); seq or graph.
  void launch_copies(int slot, void* dst, const std::vector<ShareCopy>& copies, const KernelSequence* seq,
                     hipGraphExec_t graph, bool skip_varint = false);
  // Enqueue one fan-out step (see FanoutStep).
  void launch_fanout(int slot, const FanoutStep& s);
  // Enqueue one programmed step (see StepProgram).
  // skip_varint: no request of the step has packed varint ids (see launch_seq)
  void launch_program(int slot, const StepProgram& p, const void* h2d_src, int64_t h2d_bytes,
                      bool skip_varint = false);
  // Block until the slot's last step has finished (scores are on the host).
  void wait(int slot);
  // Bounded wait: false when the step has not finished within timeout_us or a
  // communicator reports an asynchronous error (*err says which). Polls the
  // completion event (spin-yield for the first 2 ms, then 50 us sleeps) so a
  // dead peer or a stuck kernel cannot block the caller forever.
  bool wait_for(int slot, int64_t timeout_us, const std::vector<comm::RcclComm*>& comms, std::string* err);
  bool query(int slot);
  // Microseconds between the slot's last H2D start and compute end (diagnostic).
  int slots() const { return int(done_.size()); }
  int aux_cus() const { return aux_cus_; }  // CUs of the step-program aux lane (0: unmasked / not created)
  hipStream_t compute_stream() const { return compute_; }
  hipStream_t copy_stream() const { return copy_; }
  // Local steps: the launcher waits on the host for each step's H2D before it
  // enqueues the step's kernels (true), or the compute stream waits for the
  // copy's event on the device (false) - see h2d().
  void set_host_wait_h2d(bool v) { host_wait_h2d_ = v; }
  bool host_wait_h2d() const { return host_wait_h2d_; }
  // Local and programmed steps launched while earlier steps still run: a
  // feeder thread enqueues each step's kernels once the host sees its H2D
  // landed, so the compute queue carries no cross-queue wait packet (true, the
  // default), or the compute stream waits on the copy's event on the device
  // (false; always so for a step launched on an idle GPU). Set before the
  // first launch.
  void set_feed_h2d(bool v) { feed_h2d_ = v; }
  bool feed_h2d() const { return feed_h2d_; }

 private:
  int device_;
  void copy_checked(void* dst, const void* src, int64_t nbytes, hipMemcpyKind kind, hipStream_t st, int slot,
                    const char* what);
  void h2d(int slot, void* dst, const void* src, int64_t nbytes, hipStream_t consumer, bool alternate);
  void h2d_copies(int slot, void* dst, const std::vector<ShareCopy>& copies, hipStream_t consumer, bool alternate);
  hipStream_t copy2_ = nullptr;  // second H2D stream, alternated with copy_ by local steps
  // default: the device waits (round 3, one box, 3 interleaved reps of the
  // served DeepFM step with fp32-weight 5.8 MB copies: 92.5 / 94.7 / 94.7 M
  // vs host wait 89.1 / 85.4 / 97.8 M; DLRM 66.7 vs 54.3 M with 8.6 MB copies)
  bool host_wait_h2d_ = false;
  uint64_t n_h2d_ = 0;
  // host saw the slot's last step complete (set by wait/query, possibly from
  // another thread than the launcher)
  std::unique_ptr<std::atomic<bool>[]> observed_;
  void ensure_fanout_streams();
  void ensure_aux_stream(bool program);
  hipStream_t copy_ = nullptr, compute_ = nullptr, ingress_ = nullptr, egress_ = nullptr;
  std::vector<hipEvent_t> h2d_done_, done_, in_done_, fwd_done_;
  std::vector<hipEvent_t> prog_ev_;  // [slot * kProgEvents + k], created on first program launch
  int last_prog_slot_ = -1;
  int aux_cus_ = 0;  // CUs of the program aux lane's queue (0: unmasked)
  std::vector<char> used_;  // not vector<bool>: written by the launcher, read by the waiter

  // feeder (feed_h2d_): local steps whose kernels wait for their H2D on the host
  // The compute queue then holds no barrier packet in front of a step: an
  // event wait on the SDMA copy costs ~6 us of idle GPU at every step boundary
  // even when the copy landed long before (tools/native/step_gap.hip: 221.9 vs
  // 217.3 us per launch for a 216 us kernel), and a host-observed copy needs
  // none - its bytes are visible to every kernel enqueued after that.
  struct FeedJob {
    int slot = 0;
    const KernelSequence* seq = nullptr;
    hipGraphExec_t graph = nullptr;
    bool skip_varint = false;
    bool program = false;  // a programmed step (prog): its ops after the H2D
    StepProgram prog;
  };
  void program_body(int slot, const StepProgram& p, bool skip_varint, bool fed);
  // a fan-out step after its H2D: ingress (unpack + row exchange), forward on
  // the compute stream, egress (score exchange + D2H)
  void fanout_body(int slot, const FanoutStep& s);
  bool feed_h2d_ = true;
  std::thread feeder_;
  std::mutex feed_mu_;
  std::condition_variable feed_cv_;
  std::deque<FeedJob> feed_q_;
  bool feed_stop_ = false;
  std::atomic<bool> feed_failed_{false};
  std::string feed_error_;  // written once by the feeder before feed_failed_ is set
  // per slot: jobs handed to the feeder / jobs it has enqueued on the device
  std::unique_ptr<std::atomic<uint64_t>[]> queued_, launched_;
  void feed(const FeedJob& j);
  void feeder_loop();
  bool slot_launched(int slot) const {
    return launched_[slot].load(std::memory_order_acquire) == queued_[slot].load(std::memory_order_acquire);
  }
  bool want_feed(int64_t nbytes);            // feed this step: the GPU is still busy with earlier ones
  int last_slot_ = -1;                       // slot of the last launch (launcher thread)
  void wait_slot_launched(int slot) const;  // spin until the feeder enqueued the slot's last job
  void drain_feeder() const;                 // ... every slot's
};

}  // namespace runtime
}  // namespace dtfs

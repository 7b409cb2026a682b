#include "step_runner.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace dtfs {
namespace runtime {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

// Step completion is an ordinary hipEventRecord marker after the step's last
// kernel. (Round 2 measured the alternatives - device-scope release, an event
// bound to the last dispatch, no system fence - in bench/wait_gap.py; none
// paid on the served step.)
StepRunner::StepRunner(int device, int slots) : device_(device) {
  if (slots < 1) slots = 1;
  ck(hipSetDevice(device), "hipSetDevice");
  // Local steps alternate their H2D copies over two copy streams: back-to-back
  // SDMA copies on one stream leave the engine idle ~15 us between commands;
  // on two streams one copy's setup overlaps the other's transfer (8.6 MB per
  // step every ~153 us instead of ~173 us, bench/copy_pipe.py on MI355X). A
  // fan-out runner keeps one (its ingress / egress streams take the other
  // hardware queues).
  ck(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "hipStreamCreate(copy)");
  // (Round 4 A/Bs, not adopted and removed: one copy stream - no change; a
  // highest-priority compute stream - much slower, the copy and resolve queues
  // starve; profiles/r04_session2.md.)
  ck(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking), "hipStreamCreate(compute)");
  h2d_done_.resize(slots);
  done_.resize(slots);
  used_.assign(size_t(slots), 0);
  observed_.reset(new std::atomic<bool>[size_t(slots)]);
  for (int i = 0; i < slots; ++i) observed_[i].store(false);
  // Step-done events keep the system-scope release: the head kernel writes the
  // scores to pinned host memory, and only that release orders them before the
  // signal the host polls (without it +1.5 %, not adopted: profiles/r04_session2.md).
  const unsigned done_flags = hipEventDisableTiming;
  for (int i = 0; i < slots; ++i) {
    ck(hipEventCreateWithFlags(&h2d_done_[i], hipEventDisableTiming), "hipEventCreate");
    ck(hipEventCreateWithFlags(&done_[i], done_flags), "hipEventCreate");
  }
  queued_.reset(new std::atomic<uint64_t>[size_t(slots)]);
  launched_.reset(new std::atomic<uint64_t>[size_t(slots)]);
  for (int i = 0; i < slots; ++i) {
    queued_[i].store(0);
    launched_[i].store(0);
  }
  if (const char* e = std::getenv("DTFS_FEED_H2D")) feed_h2d_ = std::atoi(e) != 0;
}

StepRunner::~StepRunner() {
  if (feeder_.joinable()) {
    {
      std::lock_guard<std::mutex> lk(feed_mu_);
      feed_stop_ = true;
    }
    feed_cv_.notify_all();
    feeder_.join();
  }
  hipSetDevice(device_);
  for (hipStream_t s : {compute_, copy_, copy2_, ingress_, egress_})
    if (s) hipStreamSynchronize(s);
  for (auto* v : {&h2d_done_, &done_, &in_done_, &fwd_done_, &prog_ev_})
    for (auto e : *v) hipEventDestroy(e);
  for (hipStream_t s : {compute_, copy_, copy2_, ingress_, egress_})
    if (s) hipStreamDestroy(s);
}

void StepRunner::ensure_aux_stream(bool program) {
  if (ingress_) return;
  // A step program's aux lane (only step programs create it first; the fan-out
  // streams create it plain) runs on half of the CUs: step k+1's resolve pass
  // then leaves the other half to step k's GEMMs and head instead of taking CU
  // slots all over the chip - DeepFM 111.0 / 111.1 vs 108.9 / 108.6 M and
  // 103.0 / 103.3 vs 102.0 / 102.2 M on two boxes; 64 CUs was unstable (76.7 /
  // 106.8 M), 96 / 160 / 192 no better than none (profiles/r04_session2.md).
  // DTFS_AUX_CUS=n overrides the CU count (0: no mask).
  int n = 0;
  if (program) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_);
    n = cus >= 256 ? cus / 2 : 0;
    if (const char* e = std::getenv("DTFS_AUX_CUS")) n = std::atoi(e);
    if (n >= cus) n = 0;
  }
  if (n > 0 && n < 256) {
    uint32_t mask[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // the first n bits
    for (int i = 0; i < n; ++i) mask[i / 32] |= 1u << (i % 32);
    ck(hipExtStreamCreateWithCUMask(&ingress_, 8, mask), "hipExtStreamCreateWithCUMask(ingress)");
    aux_cus_ = n;
    return;
  }
  ck(hipStreamCreateWithFlags(&ingress_, hipStreamNonBlocking), "hipStreamCreate(ingress)");
}

void StepRunner::ensure_fanout_streams() {
  if (egress_) return;
  ensure_aux_stream(false);
  ck(hipStreamCreateWithFlags(&egress_, hipStreamNonBlocking), "hipStreamCreate(egress)");
  in_done_.resize(done_.size());
  fwd_done_.resize(done_.size());
  for (size_t i = 0; i < done_.size(); ++i) {
    ck(hipEventCreateWithFlags(&in_done_[i], hipEventDisableTiming), "hipEventCreate");
    ck(hipEventCreateWithFlags(&fwd_done_[i], hipEventDisableTiming), "hipEventCreate");
  }
}

// An async copy that fails is a server error, never retried with another
// direction: the failure record says which memory HIP saw (the round-2 retry of
// hipErrorInvalidMemcpyDirection as hipMemcpyDefault hid the cause).
void StepRunner::copy_checked(void* dst, const void* src, int64_t nbytes, hipMemcpyKind kind, hipStream_t st,
                              int slot, const char* what) {
  const hipError_t e = hipMemcpyAsync(dst, src, size_t(nbytes), kind, st);
  if (e == hipSuccess) return;
  (void)hipGetLastError();
  auto describe = [](const void* p) {
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof(at));
    const hipError_t q = hipPointerGetAttributes(&at, p);
    char buf[160];
    if (q != hipSuccess) {
      std::snprintf(buf, sizeof(buf), "%p (no HIP attributes: %s)", p, hipGetErrorString(q));
    } else {
      std::snprintf(buf, sizeof(buf), "%p (type %d, device %d, host %p, dev %p)", p, int(at.type), at.device,
                    at.hostPointer, at.devicePointer);
    }
    (void)hipGetLastError();
    return std::string(buf);
  };
  const std::string msg = std::string("hipMemcpyAsync(") + what + ", slot " + std::to_string(slot) + ", " +
                          std::to_string(nbytes) + " B): " + hipGetErrorString(e) + "; dst " + describe(dst) +
                          ", src " + describe(src);
  std::fprintf(stderr, "[step_runner] %s\n", msg.c_str());
  throw std::runtime_error(msg);
}

void StepRunner::h2d(int slot, void* dst, const void* src, int64_t nbytes, hipStream_t consumer, bool alternate) {
  std::vector<ShareCopy> one;
  if (nbytes > 0) one.push_back(ShareCopy{0, static_cast<const uint8_t*>(src), nbytes});
  h2d_copies(slot, dst, one, consumer, alternate);
}

// Feeder: local steps' kernels, enqueued in launch order once their copy landed.
void StepRunner::feed(const FeedJob& j) {
  if (!feeder_.joinable()) feeder_ = std::thread([this] { feeder_loop(); });
  queued_[j.slot].fetch_add(1, std::memory_order_acq_rel);
  {
    std::lock_guard<std::mutex> lk(feed_mu_);
    feed_q_.push_back(j);
  }
  feed_cv_.notify_one();
}

void StepRunner::feeder_loop() {
  try {
    ck(hipSetDevice(device_), "hipSetDevice(feeder)");
    for (;;) {
      FeedJob j;
      {
        std::unique_lock<std::mutex> lk(feed_mu_);
        feed_cv_.wait(lk, [&] { return feed_stop_ || !feed_q_.empty(); });
        if (feed_q_.empty()) return;  // stopping, nothing left
        j = feed_q_.front();
      }
      // the copy: spin-yield for the first 2 ms (it normally landed long ago:
      // the next step's copy runs under the current step's kernels), then
      // 20 us sleeps; the runner's destruction ends the wait
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t e = hipEventQuery(h2d_done_[j.slot]);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) ck(e, "hipEventQuery(h2d, feeder)");
        {
          std::lock_guard<std::mutex> lk(feed_mu_);
          if (feed_stop_) return;
        }
        if (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(2)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
      if (j.program) {
        program_body(j.slot, j.prog, j.skip_varint, true);
      } else if (j.seq) {
        j.seq->launch(compute_, done_[j.slot], true, j.skip_varint);
      } else {
        ck(hipGraphLaunch(j.graph, compute_), "hipGraphLaunch(feeder)");
        ck(hipEventRecord(done_[j.slot], compute_), "hipEventRecord(done, feeder)");
      }
      {
        std::lock_guard<std::mutex> lk(feed_mu_);
        feed_q_.pop_front();
      }
      launched_[j.slot].fetch_add(1, std::memory_order_acq_rel);
    }
  } catch (const std::exception& e) {
    feed_error_ = e.what();
    feed_failed_.store(true, std::memory_order_release);
    std::fprintf(stderr, "[step_runner] feeder: %s\n", e.what());
  }
}

// Feed this step (rather than enqueue it with a device-side wait) only while
// the GPU is busy with earlier steps: that is where the wait packet costs idle
// time between back-to-back steps. On an idle GPU the feeder thread's wake-up
// (a condition variable, tens of us on a loaded host) would only add latency
// to a lone request's step.
bool StepRunner::want_feed(int64_t nbytes) {
  if (!feed_h2d_ || host_wait_h2d_ || nbytes <= 0) return false;
  {
    std::lock_guard<std::mutex> lk(feed_mu_);
    if (!feed_q_.empty()) return true;  // keep launch order: behind the jobs still queued
  }
  const int last = last_slot_;
  if (last < 0 || !slot_launched(last)) return last >= 0;
  return hipEventQuery(done_[last]) == hipErrorNotReady;
}

void StepRunner::wait_slot_launched(int slot) const {
  while (!slot_launched(slot) && !feed_failed_.load(std::memory_order_acquire)) std::this_thread::yield();
}

void StepRunner::drain_feeder() const {
  for (int s = 0; s < int(done_.size()); ++s) wait_slot_launched(s);
}

void StepRunner::h2d_copies(int slot, void* dst, const std::vector<ShareCopy>& copies, hipStream_t consumer,
                            bool alternate) {
  // the slot's previous job must be on the device before its events are
  // re-recorded or waited on (the live server observed that step complete,
  // so this is normally already true)
  wait_slot_launched(slot);
  hipStream_t st = copy_;
  if (alternate) {
    if (!copy2_) ck(hipStreamCreateWithFlags(&copy2_, hipStreamNonBlocking), "hipStreamCreate(copy2)");
    if (n_h2d_++ & 1) st = copy2_;
  }
  // WAR on the slot's buffers: its previous step must have finished reading
  // them. Skipped when the host already saw that step complete (the live
  // server waits for step k - depth before it launches k).
  if (used_[slot] && !observed_[slot].load(std::memory_order_acquire))
    ck(hipStreamWaitEvent(st, done_[slot], 0), "hipStreamWaitEvent(copy)");
  int64_t nbytes = 0;
  for (const ShareCopy& c : copies) {
    if (c.n <= 0) continue;
    copy_checked(static_cast<uint8_t*>(dst) + c.dst_off, c.src, c.n, hipMemcpyHostToDevice, st, slot, "H2D");
    nbytes += c.n;
  }
  ck(hipEventRecord(h2d_done_[slot], st), "hipEventRecord(h2d)");
  if (host_wait_h2d_ && consumer == compute_ && nbytes > 0) {
    // The launcher thread waits for the copy instead of the compute queue:
    // a cross-queue barrier packet in front of every step costs ~5-7 us of
    // idle GPU at the step boundary when the copy has not landed yet
    // (tools/studies/step_timeline.py, MI355X). The price: the launcher
    // cannot issue the next step's copy while it waits, so copies never
    // overlap and a step whose copy takes longer than its kernels is
    // H2D-paced: the default is the device-side wait (step_runner.h).
    // Kernels are enqueued after the copy completed, so stream order alone is
    // enough.
    for (;;) {
      const hipError_t e = hipEventQuery(h2d_done_[slot]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) ck(e, "hipEventQuery(h2d)");
      std::this_thread::yield();
    }
  } else if (consumer) {  // null: the feeder waits for the copy on the host
    ck(hipStreamWaitEvent(consumer, h2d_done_[slot], 0), "hipStreamWaitEvent(h2d)");
  }
  observed_[slot].store(false, std::memory_order_release);
}

void StepRunner::launch_fanout(int slot, const FanoutStep& s) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (!s.cin || !s.cout || !(s.forward || s.forward_seq))
    throw std::invalid_argument("fan-out step needs both communicators and a forward");
  ck(hipSetDevice(device_), "hipSetDevice");
  ensure_fanout_streams();
  // copy (WAR on the slot's buffers), then ingress: unpack + row exchange
  // one copy stream here: with the ingress / egress streams a second one
  // shares a hardware queue (GPU_MAX_HW_QUEUES = 4) and serialises the step
  // (329 vs 187 us per step measured)
  // (fed like a local step - the feeder enqueuing the ingress once the host
  // saw the copy, on the compute stream or the ingress lane - it measured
  // slower: 109.2 / 112.0 and 105.4 vs 115.4 M with --force-fanout,
  // profiles/r06_feed_h2d.md)
  drain_feeder();
  last_slot_ = slot;
  h2d(slot, s.h2d_dst, s.h2d_src, s.h2d_bytes, ingress_, false);
  fanout_body(slot, s);
  used_[slot] = 1;
}

void StepRunner::fanout_body(int slot, const FanoutStep& s) {
  hipStream_t in = ingress_;
  if (s.ingress_seq) s.ingress_seq->launch(in, nullptr, false, s.skip_varint);
  else if (s.ingress) ck(hipGraphLaunch(s.ingress, in), "hipGraphLaunch(ingress)");
  if (s.mode == 0) s.cin->alltoall(s.send, s.recv, s.in_bytes, in);
  else s.cin->scatter(s.send, s.recv, s.in_bytes, 0, in);
  // the forward's resolve pass on this lane: step k+1's runs beside step k's forward
  if (s.resolve_seq) s.resolve_seq->launch(in);
  else if (s.resolve) ck(hipGraphLaunch(s.resolve, in), "hipGraphLaunch(resolve)");
  ck(hipEventRecord(in_done_[slot], in), "hipEventRecord(in)");
  // compute: the forward graph
  ck(hipStreamWaitEvent(compute_, in_done_[slot], 0), "hipStreamWaitEvent(compute)");
  if (s.forward_seq) {
    s.forward_seq->launch(compute_, fwd_done_[slot]);
  } else {
    ck(hipGraphLaunch(s.forward, compute_), "hipGraphLaunch(forward)");
    ck(hipEventRecord(fwd_done_[slot], compute_), "hipEventRecord(fwd)");
  }
  // egress: score exchange + D2H (SDMA)
  ck(hipStreamWaitEvent(egress_, fwd_done_[slot], 0), "hipStreamWaitEvent(egress)");
  if (s.mode == 0) s.cout->alltoall(s.scores, s.back, s.out_bytes, egress_);
  else s.cout->gather(s.scores, s.back, s.out_bytes, 0, egress_);
  if (s.d2h_bytes > 0) copy_checked(s.h_out, s.back, s.d2h_bytes, hipMemcpyDeviceToHost, egress_, slot, "D2H");
  ck(hipEventRecord(done_[slot], egress_), "hipEventRecord(done)");
}

void StepProgram::validate() const {
  if (h2d_lane != 0 && h2d_lane != 1) throw std::invalid_argument("program: h2d_lane must be 0 or 1");
  // aux-lane work (the H2D landing there counts) must be covered by an aux
  // record that the compute lane waits for, or the step could be reported done
  // while its exchange is still running
  int64_t aux_ops = h2d_lane == 1 ? 1 : 0, joined = 0;
  bool recorded[kProgEvents] = {};
  int64_t covers[kProgEvents] = {};  // aux ops before the event's record (aux lane records only)
  for (const ProgOp& o : ops) {
    if (o.lane != 0 && o.lane != 1) throw std::invalid_argument("program: lane must be 0 or 1");
    switch (o.kind) {
      case ProgOp::kKernels:
        if (!o.seq && !o.graph) throw std::invalid_argument("program: kernels op without a sequence or graph");
        break;
      case ProgOp::kAllToAll:
      case ProgOp::kAllGather:
      case ProgOp::kReduceScatter:
        if (!o.comm || !o.send || !o.recv) throw std::invalid_argument("program: collective without buffers");
        break;
      case ProgOp::kRecord:
      case ProgOp::kWait:
      case ProgOp::kWaitPrev:
        if (o.event < 0 || o.event >= kProgEvents) throw std::invalid_argument("program: event index out of range");
        break;
      default:
        throw std::invalid_argument("program: bad op kind");
    }
    if (o.kind == ProgOp::kRecord) {
      recorded[o.event] = true;
      covers[o.event] = o.lane == 1 ? aux_ops : 0;
    } else if (o.kind == ProgOp::kWait) {
      if (!recorded[o.event]) throw std::invalid_argument("program: event waited before it is recorded");
      if (o.lane == 0) joined = std::max(joined, covers[o.event]);
    } else if (o.kind != ProgOp::kWaitPrev && o.lane == 1) {
      ++aux_ops;
    }
  }
  if (joined < aux_ops) throw std::invalid_argument("program: aux-lane work is not joined into the compute lane");
}

// The step-done event rides on the step's last kernel dispatch
// (hipExtLaunchKernel stop event) instead of a separate marker packet behind
// it: one packet less at the step boundary, DeepFM 112.2 / 112.7 / 111.3 vs
// 110.4 / 110.1 / 109.7 M interleaved (profiles/r04_session2.md). The event
// keeps its system-scope release (done_ events are created without
// hipEventDisableSystemFence, and a bound event sets the scope of the command
// it is bound to), so the scores the head kernel wrote to pinned host memory
// are visible when it signals.

void StepRunner::launch_program(int slot, const StepProgram& p, const void* h2d_src, int64_t h2d_bytes,
                                bool skip_varint) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  ck(hipSetDevice(device_), "hipSetDevice");
  const bool fed = want_feed(h2d_bytes);
  last_slot_ = slot;
  if (!fed) drain_feeder();
  ensure_aux_stream(true);  // the aux lane is the ingress stream
  if (prog_ev_.empty()) {
    prog_ev_.resize(done_.size() * kProgEvents);
    // lane-to-lane dependencies stay on the device: no system-scope release
    // (a system-fenced marker between two kernels of a step measured a 7-22 us
    // bubble on MI355X, bench/step_timeline.py)
    for (auto& e : prog_ev_)
      ck(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence), "hipEventCreate(program)");
  }
  hipStream_t lanes[2] = {compute_, ingress_};
  // WAR on the slot's buffers + the H2D of the request bytes. Copies
  // alternate over two copy streams unless the fan-out streams exist too
  // (copy, copy2, compute, aux = GPU_MAX_HW_QUEUES 4; a fifth stream would
  // alias a queue and serialise the step)
  if (fed) {
    // fed like a local step: the feeder enqueues the program once the host
    // saw the copy land (program_body(fed): no lane waits just for the copy)
    h2d(slot, p.h2d_dst, h2d_src, h2d_bytes, nullptr, egress_ == nullptr);
    used_[slot] = 1;
    FeedJob j;
    j.slot = slot;
    j.skip_varint = skip_varint;
    j.program = true;
    j.prog = p;
    feed(j);
    return;
  }
  h2d(slot, p.h2d_dst, h2d_src, h2d_bytes, lanes[p.h2d_lane], egress_ == nullptr);
  program_body(slot, p, skip_varint, false);
  used_[slot] = 1;
}

void StepRunner::program_body(int slot, const StepProgram& p, bool skip_varint, bool fed) {
  hipStream_t lanes[2] = {compute_, ingress_};
  hipEvent_t* ev = &prog_ev_[size_t(slot) * kProgEvents];
  const ProgOp* last = p.ops.empty() ? nullptr : &p.ops.back();
  const bool bound = last && last->kind == ProgOp::kKernels && last->lane == 0 && last->seq;
  // fed: the copy is host-observed, so an aux-lane record with no aux work
  // before it (the lane only carried the copy) joins nothing - it and the
  // compute-lane waits on it are dropped (a cross-queue wait packet costs a
  // few us of idle GPU even when satisfied)
  bool aux_work = false, trivial[kProgEvents] = {};
  for (const ProgOp& o : p.ops) {
    hipStream_t st = lanes[o.lane];
    if (fed) {
      // (a varint-only sequence launched with skip_varint enqueues nothing)
      const bool noop = o.kind == ProgOp::kKernels && o.seq && skip_varint && o.seq->empty_without_varint();
      if (o.lane == 1 && o.kind != ProgOp::kRecord && o.kind != ProgOp::kWait && o.kind != ProgOp::kWaitPrev && !noop)
        aux_work = true;
      if (o.kind == ProgOp::kRecord && o.lane == 1 && !aux_work) {
        trivial[o.event] = true;
        continue;
      }
      if (o.kind == ProgOp::kWait && trivial[o.event]) continue;
    }
    switch (o.kind) {
      case ProgOp::kKernels:
        if (o.seq) {
          if (bound && &o == last) o.seq->launch(st, done_[slot], true, skip_varint);
          else o.seq->launch(st, nullptr, false, skip_varint);
        } else {
          ck(hipGraphLaunch(o.graph, st), "hipGraphLaunch(program)");
        }
        break;
      case ProgOp::kAllToAll:
        o.comm->alltoall(o.send, o.recv, o.bytes, st);
        break;
      case ProgOp::kAllGather:
        o.comm->allgather(o.send, o.recv, o.bytes, st);
        break;
      case ProgOp::kReduceScatter:
        o.comm->reduce_scatter_bf16(o.send, o.recv, o.bytes, st);
        break;
      case ProgOp::kRecord:
        ck(hipEventRecord(ev[o.event], st), "hipEventRecord(program)");
        break;
      case ProgOp::kWait:
        ck(hipStreamWaitEvent(st, ev[o.event], 0), "hipStreamWaitEvent(program)");
        break;
      case ProgOp::kWaitPrev:
        // the previous step recorded this event before this launch (the host
        // launches steps in order), and its slot is not reused before this one
        if (last_prog_slot_ >= 0)
          ck(hipStreamWaitEvent(st, prog_ev_[size_t(last_prog_slot_) * kProgEvents + o.event], 0),
             "hipStreamWaitEvent(program prev)");
        break;
    }
  }
  if (!bound) ck(hipEventRecord(done_[slot], compute_), "hipEventRecord(done)");
  last_prog_slot_ = slot;
}

void StepRunner::launch(int slot, void* dst, const void* src, int64_t nbytes, hipGraphExec_t graph) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  ck(hipSetDevice(device_), "hipSetDevice");
  drain_feeder();
  last_slot_ = slot;
  h2d(slot, dst, src, nbytes, compute_, true);
  ck(hipGraphLaunch(graph, compute_), "hipGraphLaunch");
  ck(hipEventRecord(done_[slot], compute_), "hipEventRecord(done)");
  used_[slot] = 1;
}

void StepRunner::launch_seq(int slot, void* dst, const void* src, int64_t nbytes, const KernelSequence* seq,
                            bool skip_varint) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (!seq) throw std::invalid_argument("null kernel sequence");
  ck(hipSetDevice(device_), "hipSetDevice");
  const bool fed = want_feed(nbytes);
  last_slot_ = slot;
  if (fed) {
    h2d(slot, dst, src, nbytes, nullptr, true);
    used_[slot] = 1;
    feed(FeedJob{slot, seq, nullptr, skip_varint});
    return;
  }
  drain_feeder();  // keep launch order on the compute stream
  h2d(slot, dst, src, nbytes, compute_, true);
  seq->launch(compute_, done_[slot], true, skip_varint);
  used_[slot] = 1;
}

void StepRunner::launch_copies(int slot, void* dst, const std::vector<ShareCopy>& copies, const KernelSequence* seq,
                               hipGraphExec_t graph, bool skip_varint) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (!seq && !graph) throw std::invalid_argument("launch_copies: no kernel sequence or graph");
  ck(hipSetDevice(device_), "hipSetDevice");
  int64_t nbytes = 0;
  for (const ShareCopy& c : copies) nbytes += c.n > 0 ? c.n : 0;
  const bool fed = want_feed(nbytes);
  last_slot_ = slot;
  if (fed) {
    h2d_copies(slot, dst, copies, nullptr, true);
    used_[slot] = 1;
    feed(FeedJob{slot, seq, seq ? nullptr : graph, skip_varint});
    return;
  }
  drain_feeder();
  h2d_copies(slot, dst, copies, compute_, true);
  if (seq) {
    seq->launch(compute_, done_[slot], true, skip_varint);
  } else {
    ck(hipGraphLaunch(graph, compute_), "hipGraphLaunch");
    ck(hipEventRecord(done_[slot], compute_), "hipEventRecord(done)");
  }
  used_[slot] = 1;
}

void StepRunner::wait(int slot) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  wait_slot_launched(slot);
  if (feed_failed_.load(std::memory_order_acquire)) throw std::runtime_error("step feeder: " + feed_error_);
  if (used_[slot]) ck(hipEventSynchronize(done_[slot]), "hipEventSynchronize");
  observed_[slot].store(true, std::memory_order_release);
}

bool StepRunner::wait_for(int slot, int64_t timeout_us, const std::vector<comm::RcclComm*>& comms,
                          std::string* err) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto last_comm_check = t0;
  if (used_[slot]) {
    for (;;) {
      if (feed_failed_.load(std::memory_order_acquire)) {
        *err = "step feeder: " + feed_error_;
        return false;
      }
      // a job still with the feeder has not recorded its done event yet
      const hipError_t e = slot_launched(slot) ? hipEventQuery(done_[slot]) : hipErrorNotReady;
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) {
        *err = std::string("hipEventQuery: ") + hipGetErrorString(e);
        return false;
      }
      const auto now = clk::now();
      const int64_t el = std::chrono::duration_cast<std::chrono::microseconds>(now - t0).count();
      if (el > timeout_us) {
        *err = "step not finished after " + std::to_string(el / 1000) + " ms";
        return false;
      }
      if (!comms.empty() && now - last_comm_check > std::chrono::milliseconds(1)) {
        last_comm_check = now;
        for (auto* c : comms) {
          if (!c) continue;
          std::string ce = c->async_error();
          if (!ce.empty()) {
            *err = "RCCL: " + ce;
            return false;
          }
        }
      }
      if (el < 2000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  // the step finished - but a peer exchange that timed out also finishes
  // (its kernel exits), so a step is only done if no communicator failed
  for (auto* c : comms) {
    if (!c) continue;
    std::string ce = c->async_error();
    if (!ce.empty()) {
      *err = "RCCL: " + ce;
      return false;
    }
  }
  observed_[slot].store(true, std::memory_order_release);
  return true;
}

bool StepRunner::query(int slot) {
  if (!used_[slot]) return true;
  if (!slot_launched(slot)) {
    if (feed_failed_.load(std::memory_order_acquire)) throw std::runtime_error("step feeder: " + feed_error_);
    return false;
  }
  hipError_t e = hipEventQuery(done_[slot]);
  if (e == hipErrorNotReady) return false;
  ck(e, "hipEventQuery");
  observed_[slot].store(true, std::memory_order_release);
  return true;
}

}  // namespace runtime
}  // namespace dtfs

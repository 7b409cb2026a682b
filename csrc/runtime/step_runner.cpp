#include "step_runner.h"

#include <stdexcept>
#include <string>

namespace dtfs {
namespace runtime {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

StepRunner::StepRunner(int device, int slots) : device_(device) {
  if (slots < 1) slots = 1;
  ck(hipSetDevice(device), "hipSetDevice");
  ck(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking), "hipStreamCreate(copy)");
  ck(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking), "hipStreamCreate(compute)");
  h2d_done_.resize(slots);
  done_.resize(slots);
  used_.assign(slots, false);
  for (int i = 0; i < slots; ++i) {
    ck(hipEventCreateWithFlags(&h2d_done_[i], hipEventDisableTiming), "hipEventCreate");
    ck(hipEventCreateWithFlags(&done_[i], hipEventDisableTiming), "hipEventCreate");
  }
}

StepRunner::~StepRunner() {
  hipSetDevice(device_);
  for (hipStream_t s : {compute_, copy_, ingress_, egress_})
    if (s) hipStreamSynchronize(s);
  for (auto* v : {&h2d_done_, &done_, &in_done_, &fwd_done_})
    for (auto e : *v) hipEventDestroy(e);
  for (hipStream_t s : {compute_, copy_, ingress_, egress_})
    if (s) hipStreamDestroy(s);
}

void StepRunner::ensure_fanout_streams() {
  if (ingress_) return;
  ck(hipStreamCreateWithFlags(&ingress_, hipStreamNonBlocking), "hipStreamCreate(ingress)");
  ck(hipStreamCreateWithFlags(&egress_, hipStreamNonBlocking), "hipStreamCreate(egress)");
  in_done_.resize(done_.size());
  fwd_done_.resize(done_.size());
  for (size_t i = 0; i < done_.size(); ++i) {
    ck(hipEventCreateWithFlags(&in_done_[i], hipEventDisableTiming), "hipEventCreate");
    ck(hipEventCreateWithFlags(&fwd_done_[i], hipEventDisableTiming), "hipEventCreate");
  }
}

void StepRunner::launch_fanout(int slot, const FanoutStep& s) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (!s.cin || !s.cout || !(s.forward || s.forward_seq))
    throw std::invalid_argument("fan-out step needs both communicators and a forward");
  ck(hipSetDevice(device_), "hipSetDevice");
  ensure_fanout_streams();
  // copy: WAR on the slot's buffers (its previous step is entirely done)
  if (used_[slot]) ck(hipStreamWaitEvent(copy_, done_[slot], 0), "hipStreamWaitEvent(copy)");
  if (s.h2d_bytes > 0)
    ck(hipMemcpyAsync(s.h2d_dst, s.h2d_src, size_t(s.h2d_bytes), hipMemcpyHostToDevice, copy_), "hipMemcpyAsync(H2D)");
  ck(hipEventRecord(h2d_done_[slot], copy_), "hipEventRecord(h2d)");
  // ingress: unpack + row exchange, off the compute stream
  ck(hipStreamWaitEvent(ingress_, h2d_done_[slot], 0), "hipStreamWaitEvent(ingress)");
  if (s.ingress_seq) s.ingress_seq->launch(ingress_);
  else if (s.ingress) ck(hipGraphLaunch(s.ingress, ingress_), "hipGraphLaunch(ingress)");
  if (s.mode == 0) s.cin->alltoall(s.send, s.recv, s.in_bytes, ingress_);
  else s.cin->scatter(s.send, s.recv, s.in_bytes, 0, ingress_);
  ck(hipEventRecord(in_done_[slot], ingress_), "hipEventRecord(in)");
  // compute: the forward graph
  ck(hipStreamWaitEvent(compute_, in_done_[slot], 0), "hipStreamWaitEvent(compute)");
  if (s.forward_seq) s.forward_seq->launch(compute_);
  else ck(hipGraphLaunch(s.forward, compute_), "hipGraphLaunch(forward)");
  ck(hipEventRecord(fwd_done_[slot], compute_), "hipEventRecord(fwd)");
  // egress: score exchange + D2H (SDMA)
  ck(hipStreamWaitEvent(egress_, fwd_done_[slot], 0), "hipStreamWaitEvent(egress)");
  if (s.mode == 0) s.cout->alltoall(s.scores, s.back, s.out_bytes, egress_);
  else s.cout->gather(s.scores, s.back, s.out_bytes, 0, egress_);
  if (s.d2h_bytes > 0)
    ck(hipMemcpyAsync(s.h_out, s.back, s.d2h_bytes, hipMemcpyDeviceToHost, egress_), "hipMemcpyAsync(D2H)");
  ck(hipEventRecord(done_[slot], egress_), "hipEventRecord(done)");
  used_[slot] = true;
}

void StepRunner::launch(int slot, void* dst, const void* src, int64_t nbytes, hipGraphExec_t graph) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  ck(hipSetDevice(device_), "hipSetDevice");
  // WAR: the previous step on this slot must have finished reading dst (its
  // graph ends after the forward), so wait for its completion event.
  if (used_[slot]) ck(hipStreamWaitEvent(copy_, done_[slot], 0), "hipStreamWaitEvent(copy)");
  if (nbytes > 0) ck(hipMemcpyAsync(dst, src, size_t(nbytes), hipMemcpyHostToDevice, copy_), "hipMemcpyAsync(H2D)");
  ck(hipEventRecord(h2d_done_[slot], copy_), "hipEventRecord(h2d)");
  ck(hipStreamWaitEvent(compute_, h2d_done_[slot], 0), "hipStreamWaitEvent(compute)");
  ck(hipGraphLaunch(graph, compute_), "hipGraphLaunch");
  ck(hipEventRecord(done_[slot], compute_), "hipEventRecord(done)");
  used_[slot] = true;
}

void StepRunner::launch_seq(int slot, void* dst, const void* src, int64_t nbytes, const KernelSequence* seq) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (!seq) throw std::invalid_argument("null kernel sequence");
  ck(hipSetDevice(device_), "hipSetDevice");
  if (used_[slot]) ck(hipStreamWaitEvent(copy_, done_[slot], 0), "hipStreamWaitEvent(copy)");
  if (nbytes > 0) ck(hipMemcpyAsync(dst, src, size_t(nbytes), hipMemcpyHostToDevice, copy_), "hipMemcpyAsync(H2D)");
  ck(hipEventRecord(h2d_done_[slot], copy_), "hipEventRecord(h2d)");
  ck(hipStreamWaitEvent(compute_, h2d_done_[slot], 0), "hipStreamWaitEvent(compute)");
  seq->launch(compute_);
  ck(hipEventRecord(done_[slot], compute_), "hipEventRecord(done)");
  used_[slot] = true;
}

void StepRunner::wait(int slot) {
  if (slot < 0 || slot >= int(done_.size())) throw std::out_of_range("slot");
  if (used_[slot]) ck(hipEventSynchronize(done_[slot]), "hipEventSynchronize");
}

bool StepRunner::query(int slot) {
  if (!used_[slot]) return true;
  hipError_t e = hipEventQuery(done_[slot]);
  if (e == hipErrorNotReady) return false;
  ck(e, "hipEventQuery");
  return true;
}

}  // namespace runtime
}  // namespace dtfs

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
  if (compute_) hipStreamSynchronize(compute_);
  if (copy_) hipStreamSynchronize(copy_);
  for (auto e : h2d_done_) hipEventDestroy(e);
  for (auto e : done_) hipEventDestroy(e);
  if (copy_) hipStreamDestroy(copy_);
  if (compute_) hipStreamDestroy(compute_);
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

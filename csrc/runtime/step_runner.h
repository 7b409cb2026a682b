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

#include <cstdint>
#include <vector>

namespace dtfs {
namespace runtime {

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
  // Block until the slot's last step has finished (scores are on the host).
  void wait(int slot);
  bool query(int slot);
  // Microseconds between the slot's last H2D start and compute end (diagnostic).
  int slots() const { return int(done_.size()); }
  hipStream_t compute_stream() const { return compute_; }
  hipStream_t copy_stream() const { return copy_; }

 private:
  int device_;
  hipStream_t copy_ = nullptr, compute_ = nullptr;
  std::vector<hipEvent_t> h2d_done_, done_;
  std::vector<bool> used_;
};

}  // namespace runtime
}  // namespace dtfs

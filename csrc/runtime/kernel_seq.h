// KernelSequence: a captured HIP graph replayed as plain stream launches.
//
// Measured on MI355X (bench/graph_gap.py, DeepFM step at 8192 rows): replaying
// the step graph back-to-back leaves ~8.5 us idle between graphs (~13.7 us when
// each launch waits on an event of the H2D stream), while the same kernels
// launched eagerly run back-to-back with no gap - 11 us of a ~115 us step. The
// serving loop launches from a C++ thread that runs several steps ahead, so the
// per-kernel host cost of direct launches is hidden and the graph buys nothing.
//
// The model is still captured once through PyTorch (torch.cuda.CUDAGraph,
// keep_graph=True), which fixes every kernel's arguments and buffers; this
// class walks the captured graph in dependency order and keeps each node's
// launch parameters (owned by the graph, which must outlive the sequence).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

namespace dtfs {
namespace runtime {

class KernelSequence {
 public:
  explicit KernelSequence(hipGraph_t graph);
  // Enqueue every node on `st`, in dependency order. With `done`, the event
  // completes with the last node: bound to the last kernel's own dispatch
  // (hipExtLaunchKernel stop event) when `bind` is set and the last node is a
  // kernel, otherwise recorded after it.
  // skip_varint: leave out the arena varint-decode kernel (the host parse
  // found no packed varint ids in this step's requests).
  void launch(hipStream_t st, hipEvent_t done = nullptr, bool bind = false, bool skip_varint = false) const;
  int size() const { return int(ops_.size()); }
  // launching it with skip_varint enqueues nothing (the sequence is only the
  // arena varint-decode kernel, or empty)
  bool empty_without_varint() const {
    for (const Op& o : ops_)
      if (!o.varint) return false;
    return true;
  }
  std::string describe() const;

 private:
  struct Op {
    int kind = 0;  // 0 kernel, 1 memcpy, 2 memset
    bool varint = false;
    hipKernelNodeParams k{};
    hipMemcpy3DParms mc{};
    hipMemsetParams ms{};
  };
  std::vector<Op> ops_;
};

}  // namespace runtime
}  // namespace dtfs

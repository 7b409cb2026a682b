#include "kernel_seq.h"

#include <hip/hip_ext.h>

#include "../kernels/launchers.h"

#include <map>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace dtfs {
namespace runtime {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace

KernelSequence::KernelSequence(hipGraph_t graph) {
  if (!graph) throw std::invalid_argument("null graph");
  size_t n = 0;
  ck(hipGraphGetNodes(graph, nullptr, &n), "hipGraphGetNodes");
  std::vector<hipGraphNode_t> nodes(n);
  ck(hipGraphGetNodes(graph, nodes.data(), &n), "hipGraphGetNodes");
  std::map<hipGraphNode_t, size_t> index;
  for (size_t i = 0; i < n; ++i) index[nodes[i]] = i;
  // Kahn's algorithm, ties broken by node order (= capture order)
  std::vector<std::vector<size_t>> users(n);
  std::vector<int> indeg(n, 0);
  for (size_t i = 0; i < n; ++i) {
    size_t nd = 0;
    ck(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd), "hipGraphNodeGetDependencies");
    std::vector<hipGraphNode_t> deps(nd);
    if (nd) ck(hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd), "hipGraphNodeGetDependencies");
    for (auto d : deps) {
      users[index.at(d)].push_back(i);
      ++indeg[i];
    }
  }
  std::vector<size_t> order;
  std::vector<char> done(n, 0);
  while (order.size() < n) {
    size_t pick = n;
    for (size_t i = 0; i < n; ++i)
      if (!done[i] && indeg[i] == 0) {
        pick = i;
        break;
      }
    if (pick == n) throw std::runtime_error("graph has a cycle");
    done[pick] = 1;
    order.push_back(pick);
    for (size_t u : users[pick]) --indeg[u];
  }
  for (size_t i : order) {
    hipGraphNodeType t;
    ck(hipGraphNodeGetType(nodes[i], &t), "hipGraphNodeGetType");
    Op op;
    if (t == hipGraphNodeTypeKernel) {
      op.kind = 0;
      ck(hipGraphKernelNodeGetParams(nodes[i], &op.k), "hipGraphKernelNodeGetParams");
      if (!op.k.kernelParams) throw std::runtime_error("kernel node without kernelParams (extra-style launch)");
      op.varint = op.k.func == arena_varint_kernel_fn();
    } else if (t == hipGraphNodeTypeMemcpy) {
      op.kind = 1;
      ck(hipGraphMemcpyNodeGetParams(nodes[i], &op.mc), "hipGraphMemcpyNodeGetParams");
      const hipMemcpy3DParms& c = op.mc;
      if (c.srcArray || c.dstArray || c.extent.height > 1 || c.extent.depth > 1 || !c.srcPtr.ptr || !c.dstPtr.ptr)
        throw std::runtime_error("unsupported memcpy node (not a plain 1-D copy)");
    } else if (t == hipGraphNodeTypeMemset) {
      op.kind = 2;
      ck(hipGraphMemsetNodeGetParams(nodes[i], &op.ms), "hipGraphMemsetNodeGetParams");
      if (op.ms.height > 1 || (op.ms.elementSize != 1 && op.ms.elementSize != 2 && op.ms.elementSize != 4))
        throw std::runtime_error("unsupported memset node");
    } else if (t == hipGraphNodeTypeEmpty) {
      continue;
    } else {
      throw std::runtime_error("unsupported graph node type " + std::to_string(int(t)));
    }
    ops_.push_back(op);
  }
}

void KernelSequence::launch(hipStream_t st, hipEvent_t done, bool bind, bool skip_varint) const {
  // a sequence that is only the varint decode (a step program's own op) is
  // skipped whole: an empty launch of it still queued behind the running
  // GEMM for a CU slot (57 us per step on the aux lane, MI355X)
  const bool skip_last = skip_varint && !ops_.empty() && ops_.back().varint;
  const bool bind_last = done && bind && !ops_.empty() && ops_.back().kind == 0 && !skip_last;
  for (size_t i = 0; i < ops_.size(); ++i) {
    const Op& op = ops_[i];
    if (skip_varint && op.varint) continue;
    if (op.kind == 0) {
      if (bind_last && i + 1 == ops_.size())
        ck(hipExtLaunchKernel(op.k.func, op.k.gridDim, op.k.blockDim, op.k.kernelParams, op.k.sharedMemBytes, st,
                              nullptr, done, 0),
           "hipExtLaunchKernel");
      else
        ck(hipLaunchKernel(op.k.func, op.k.gridDim, op.k.blockDim, op.k.kernelParams, op.k.sharedMemBytes, st),
           "hipLaunchKernel");
    } else if (op.kind == 1) {
      // a captured 1-D hipMemcpyAsync (checked at construction)
      const hipMemcpy3DParms& c = op.mc;
      const char* src = static_cast<const char*>(c.srcPtr.ptr) + c.srcPos.x;
      char* dst = static_cast<char*>(c.dstPtr.ptr) + c.dstPos.x;
      const hipError_t e = hipMemcpyAsync(dst, src, c.extent.width, c.kind, st);
      if (e != hipSuccess) {
        // fail with what HIP thinks both pointers are (never retried with
        // another direction: that would hide the cause)
        (void)hipGetLastError();
        hipPointerAttribute_t ad, as;
        std::memset(&ad, 0, sizeof(ad));
        std::memset(&as, 0, sizeof(as));
        const hipError_t qd = hipPointerGetAttributes(&ad, dst), qs = hipPointerGetAttributes(&as, src);
        (void)hipGetLastError();
        char buf[256];
        std::snprintf(buf, sizeof(buf), "replayed hipMemcpyAsync(kind %d, %zu B): %s; dst %p type %d (%s), src %p type %d (%s)",
                      int(c.kind), size_t(c.extent.width), hipGetErrorString(e), static_cast<void*>(dst), int(ad.type),
                      hipGetErrorString(qd), static_cast<const void*>(src), int(as.type), hipGetErrorString(qs));
        std::fprintf(stderr, "[kernel_seq] %s\n", buf);
        throw std::runtime_error(buf);
      }
    } else {
      const hipMemsetParams& m = op.ms;
      if (m.elementSize == 1) ck(hipMemsetD8Async(hipDeviceptr_t(m.dst), uint8_t(m.value), m.width, st), "memset");
      else if (m.elementSize == 2)
        ck(hipMemsetD16Async(hipDeviceptr_t(m.dst), uint16_t(m.value), m.width, st), "memset");
      else ck(hipMemsetD32Async(hipDeviceptr_t(m.dst), int(m.value), m.width, st), "memset");
    }
  }
  if (done && !bind_last) ck(hipEventRecord(done, st), "hipEventRecord");
}

std::string KernelSequence::describe() const {
  std::string s;
  for (const Op& op : ops_) {
    if (!s.empty()) s += ", ";
    if (op.kind == 0)
      s += "kernel<" + std::to_string(op.k.gridDim.x) + "x" + std::to_string(op.k.blockDim.x) + ">";
    else s += op.kind == 1 ? "memcpy" : "memset";
  }
  return s;
}

}  // namespace runtime
}  // namespace dtfs

// roctx ranges for the host runtime (NVTX-equivalent ranges
// around decode / H2D / compute / collectives / D2H / encode).
//
// Off unless DTFS_TRACE=1: then librocprofiler-sdk-roctx is dlopen'ed and every
// Range below becomes a roctx range that `rocprofv3 --marker-trace` records
// next to the kernel trace. When off a Range costs one branch.
#pragma once

namespace dtfs {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

struct Range {
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace dtfs

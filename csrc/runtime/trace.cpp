#include "trace.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace dtfs {
namespace trace {

namespace {
using PushFn = int (*)(const char*);
using PopFn = int (*)();
using MarkFn = void (*)(const char*);

struct Api {
  bool on = false;
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
};

const Api& api() {
  static Api a;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("DTFS_TRACE");
    if (!e || std::strcmp(e, "1") != 0) return;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    a.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
    a.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
    a.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
    a.on = a.push && a.pop;
  });
  return a;
}
}  // namespace

bool enabled() { return api().on; }

void push(const char* name) {
  const Api& a = api();
  if (a.on) a.push(name);
}

void pop() {
  const Api& a = api();
  if (a.on) a.pop();
}

void mark(const char* name) {
  const Api& a = api();
  if (a.on && a.mark) a.mark(name);
}

}  // namespace trace
}  // namespace dtfs

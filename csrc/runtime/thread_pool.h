// Small persistent fork-join pool for host-side request decode / encode.
//
// parallel_for(n, fn) runs fn(0..n-1) on the pool's workers plus the calling
// thread and returns when all items are done. Workers spin briefly before
// sleeping so back-to-back batches (one every ~100 us) do not pay a futex wake
// per item. No Python, no GIL: callers release the GIL around it.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dtfs {
namespace runtime {

class ThreadPool {
 public:
  explicit ThreadPool(int threads);
  ~ThreadPool();
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  int size() const { return int(workers_.size()) + 1; }
  void parallel_for(int64_t n, const std::function<void(int64_t)>& fn);

  // Process-wide pool (size from DTFS_HOST_THREADS, default min(8, hw threads)).
  static ThreadPool& global();

 private:
  void worker_loop();
  void drain(const std::function<void(int64_t)>& fn, int64_t n);

  std::vector<std::thread> workers_;
  std::mutex mu_;        // serialises parallel_for callers
  std::mutex wake_mu_;
  std::condition_variable wake_cv_;
  std::atomic<uint64_t> epoch_{0};
  std::atomic<bool> stop_{false};
  // the current round (guarded by wake_mu_): a worker joins only an open round,
  // copying fn_ / n_ and counting itself in active_ under the lock, so the
  // caller can close a round (and set up the next) once active_ is back to 0
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  bool open_ = false;
  std::atomic<int64_t> next_{0};
  std::atomic<int64_t> done_{0};
  std::atomic<int> active_{0};
};

}  // namespace runtime
}  // namespace dtfs

#include "thread_pool.h"

#include <algorithm>
#include <cstdlib>

namespace dtfs {
namespace runtime {

ThreadPool::ThreadPool(int threads) {
  const int extra = std::max(0, threads - 1);
  workers_.reserve(extra);
  for (int i = 0; i < extra; ++i) workers_.emplace_back([this] { worker_loop(); });
}

ThreadPool::~ThreadPool() {
  stop_.store(true);
  {
    std::lock_guard<std::mutex> lk(wake_mu_);
    epoch_.fetch_add(1);
  }
  wake_cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::drain(const std::function<void(int64_t)>& fn, int64_t n) {
  for (;;) {
    const int64_t i = next_.fetch_add(1, std::memory_order_relaxed);
    if (i >= n) break;
    fn(i);
    done_.fetch_add(1, std::memory_order_acq_rel);
  }
}

void ThreadPool::worker_loop() {
  uint64_t seen = 0;
  for (;;) {
    // spin a little on the epoch, then sleep until a new one
    int spins = 0;
    while (epoch_.load(std::memory_order_acquire) == seen && !stop_.load()) {
      if (++spins > 20000) break;
    }
    const std::function<void(int64_t)>* fn = nullptr;
    int64_t n = 0;
    {
      std::unique_lock<std::mutex> lk(wake_mu_);
      wake_cv_.wait(lk, [&] { return epoch_.load() != seen || stop_.load(); });
      if (stop_.load()) return;
      seen = epoch_.load();
      if (!open_) continue;  // woke after the round closed: nothing left to join
      fn = fn_;
      n = n_;
      active_.fetch_add(1, std::memory_order_acq_rel);
    }
    drain(*fn, n);
    active_.fetch_sub(1, std::memory_order_acq_rel);
  }
}

void ThreadPool::parallel_for(int64_t n, const std::function<void(int64_t)>& fn) {
  if (n <= 0) return;
  if (workers_.empty() || n == 1) {
    for (int64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  std::lock_guard<std::mutex> guard(mu_);
  {
    std::lock_guard<std::mutex> lk(wake_mu_);
    fn_ = &fn;
    n_ = n;
    done_.store(0, std::memory_order_relaxed);
    next_.store(0, std::memory_order_relaxed);
    open_ = true;
    epoch_.fetch_add(1, std::memory_order_acq_rel);
  }
  wake_cv_.notify_all();
  drain(fn, n);
  while (done_.load(std::memory_order_acquire) < n) std::this_thread::yield();
  {
    std::lock_guard<std::mutex> lk(wake_mu_);
    open_ = false;  // no worker joins any more; the ones inside finish their claims
    fn_ = nullptr;
  }
  // fn must outlive every worker still between its last claim and leaving drain()
  while (active_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
}

ThreadPool& ThreadPool::global() {
  static ThreadPool* pool = [] {
    int n = 0;
    if (const char* e = std::getenv("DTFS_HOST_THREADS")) n = std::atoi(e);
    if (n <= 0) n = std::min(8, int(std::max(1u, std::thread::hardware_concurrency())));
    return new ThreadPool(n);
  }();
  return *pool;
}

}  // namespace runtime
}  // namespace dtfs

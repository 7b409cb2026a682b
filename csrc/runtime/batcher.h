// Dynamic-batching queue core (the TF-Serving server-side batching the
// reference relies on, reference README.md:5,9, re-done for a GPU shard).
//
// Requests are admitted as (ticket, rows, deadline). A consumer thread calls
// next_batch(), which blocks until
//   * the queued rows reach max_batch_rows (a full batch), or
//   * the oldest queued request has waited batch_timeout_us, or
//   * the queue is closed.
// Requests are never split; one larger than max_batch_rows is served alone.
// Requests whose deadline has passed before they are batched are returned in
// the `expired` list so the caller can fail them with DEADLINE_EXCEEDED instead
// of spending GPU time on them. All waiting happens with the GIL released.
#pragma once

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <vector>

namespace dtfs {
namespace runtime {

struct BatchItem {
  int64_t ticket;
  int64_t rows;
  int64_t enqueue_us;
  int64_t deadline_us;  // 0 = none
};

struct Batch {
  std::vector<BatchItem> items;
  std::vector<BatchItem> expired;
  int64_t rows = 0;
  bool closed = false;
};

struct BatcherStats {
  int64_t submitted = 0;
  int64_t rejected = 0;
  int64_t batches = 0;
  int64_t batched_rows = 0;
  int64_t expired = 0;
  int64_t full_batches = 0;
  int64_t timeout_batches = 0;
};

int64_t now_us();

class DynamicBatcher {
 public:
  DynamicBatcher(int64_t max_batch_rows, int64_t batch_timeout_us, int64_t max_queued_rows);

  // False when the queue is closed or would exceed max_queued_rows
  // (backpressure: the caller answers RESOURCE_EXHAUSTED / UNAVAILABLE).
  bool submit(int64_t ticket, int64_t rows, int64_t deadline_us);

  // Blocks up to wait_us (<0: forever) for a batch. An empty batch with
  // closed=false means the wait timed out with nothing queued.
  // eager=true: take whatever is queued as soon as anything is (the caller's
  // device is idle, so waiting for the batch timeout only adds latency).
  Batch next_batch(int64_t wait_us, bool eager = false);

  void close();
  bool closed() const;
  int64_t queued_rows() const;
  BatcherStats stats() const;

  int64_t max_batch_rows() const { return max_batch_rows_; }
  int64_t batch_timeout_us() const { return timeout_us_; }

 private:
  const int64_t max_batch_rows_;
  const int64_t timeout_us_;
  const int64_t max_queued_rows_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<BatchItem> q_;
  int64_t queued_rows_ = 0;
  bool closed_ = false;
  BatcherStats stats_;
};

}  // namespace runtime
}  // namespace dtfs

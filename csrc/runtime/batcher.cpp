#include "batcher.h"

namespace dtfs {
namespace runtime {

int64_t now_us() {
  using namespace std::chrono;
  return duration_cast<microseconds>(steady_clock::now().time_since_epoch()).count();
}

DynamicBatcher::DynamicBatcher(int64_t max_batch_rows, int64_t batch_timeout_us, int64_t max_queued_rows)
    : max_batch_rows_(max_batch_rows > 0 ? max_batch_rows : 1),
      timeout_us_(batch_timeout_us >= 0 ? batch_timeout_us : 0),
      max_queued_rows_(max_queued_rows > 0 ? max_queued_rows : (int64_t(1) << 62)) {}

bool DynamicBatcher::submit(int64_t ticket, int64_t rows, int64_t deadline_us) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (closed_ || (queued_rows_ > 0 && queued_rows_ + rows > max_queued_rows_)) {
      ++stats_.rejected;
      return false;
    }
    q_.push_back(BatchItem{ticket, rows, now_us(), deadline_us});
    queued_rows_ += rows;
    ++stats_.submitted;
  }
  cv_.notify_one();
  return true;
}

Batch DynamicBatcher::next_batch(int64_t wait_us, bool eager) {
  Batch b;
  std::unique_lock<std::mutex> lk(mu_);
  const int64_t give_up = wait_us < 0 ? -1 : now_us() + wait_us;
  for (;;) {
    // Drop expired heads first.
    const int64_t t = now_us();
    while (!q_.empty() && q_.front().deadline_us > 0 && q_.front().deadline_us <= t) {
      b.expired.push_back(q_.front());
      queued_rows_ -= q_.front().rows;
      ++stats_.expired;
      q_.pop_front();
    }
    if (!q_.empty()) {
      const bool full = queued_rows_ >= max_batch_rows_;
      const int64_t ready_at = q_.front().enqueue_us + timeout_us_;
      if (full || eager || t >= ready_at || closed_) {
        // Take whole requests until the next one would overflow the batch.
        while (!q_.empty()) {
          const BatchItem& it = q_.front();
          if (!b.items.empty() && b.rows + it.rows > max_batch_rows_) break;
          if (it.deadline_us > 0 && it.deadline_us <= t) {
            b.expired.push_back(it);
            ++stats_.expired;
          } else {
            b.items.push_back(it);
            b.rows += it.rows;
          }
          queued_rows_ -= it.rows;
          q_.pop_front();
        }
        if (!b.items.empty()) {
          ++stats_.batches;
          stats_.batched_rows += b.rows;
          if (full) ++stats_.full_batches;
          else ++stats_.timeout_batches;
        }
        return b;
      }
      if (!b.expired.empty()) return b;
      // Wait for more work or the oldest request's timeout.
      int64_t until = ready_at;
      if (give_up >= 0 && give_up < until) until = give_up;
      if (give_up >= 0 && t >= give_up) return b;
      cv_.wait_for(lk, std::chrono::microseconds(until - t));
      continue;
    }
    if (closed_) {
      b.closed = true;
      return b;
    }
    if (!b.expired.empty()) return b;
    if (give_up >= 0) {
      if (t >= give_up) return b;
      cv_.wait_for(lk, std::chrono::microseconds(give_up - t));
    } else {
      cv_.wait(lk);
    }
  }
}

void DynamicBatcher::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    closed_ = true;
  }
  cv_.notify_all();
}

bool DynamicBatcher::closed() const {
  std::lock_guard<std::mutex> lk(mu_);
  return closed_;
}

int64_t DynamicBatcher::queued_rows() const {
  std::lock_guard<std::mutex> lk(mu_);
  return queued_rows_;
}

BatcherStats DynamicBatcher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

}  // namespace runtime
}  // namespace dtfs

#include "loadgen.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <random>
#include <stdexcept>
#include <thread>

#include "batcher.h"  // now_us()

namespace dtfs {
namespace runtime {

namespace {

// Work queue of (request index, scheduled send time) handed to submitters.
struct WorkQ {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<int64_t, int64_t>> q;
  bool stop = false;

  void push(int64_t i, int64_t t) {
    {
      std::lock_guard<std::mutex> lk(mu);
      q.emplace_back(i, t);
    }
    cv.notify_one();
  }
  bool pop(std::pair<int64_t, int64_t>* out) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return stop || !q.empty(); });
    if (q.empty()) return false;
    *out = q.front();
    q.pop_front();
    return true;
  }
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
  }
};

}  // namespace

LoadResult run_load(LiveServer& srv, const std::vector<std::string>& reqs, const LoadSpec& spec) {
  if (reqs.empty()) throw std::invalid_argument("no requests");
  if (spec.count <= 0) throw std::invalid_argument("count must be > 0");
  const bool open_loop = spec.qps > 0;
  const int C = std::max(1, spec.concurrency);
  const int64_t tail = open_loop ? 0 : (spec.tail < 0 ? C : spec.tail);
  const int64_t total = spec.warmup + spec.count + tail;
  const int64_t P = int64_t(reqs.size());

  LoadResult res;
  std::mutex mu;
  std::condition_variable cv_all;
  int64_t completed = 0;
  double t_open = 0, t_close = 0;
  std::vector<double> lat_sched;  // open loop: by request index
  std::vector<Stages> stg_sched;
  if (open_loop) {
    lat_sched.assign(size_t(spec.warmup + spec.count), -1.0);
    stg_sched.assign(size_t(spec.warmup + spec.count), Stages{});
  }
  res.latency_us.reserve(size_t(spec.count));
  WorkQ work;
  std::atomic<int64_t> next{0};

  // Every completion callback runs on a LiveServer thread (the completer, or
  // the submitter for a rejected request) and touches this frame's state
  // (mu, next, work, res). The waiter below returns - destroying all of it -
  // only once every callback has finished with it: `running` counts callbacks
  // between their first and last critical section, and the waiter needs
  // completed == total AND running == 0. (Round 3's version released mu and
  // then did next.fetch_add / work.push: the waiter could wake in between and
  // return, a use-after-return on the completer thread.)
  int running = 0;
  auto on_done = [&](int64_t i, int64_t t_sched, int64_t t_pop, Reply&& r) {
    const int64_t t = now_us();
    Stages sg{};
    if (r.code == kOk && r.t_arrive > 0 && r.t_encoded > 0) {
      sg = {float(t_pop - t_sched), float(r.t_arrive - t_pop), float(r.t_launch - r.t_arrive),
            float(r.t_done - r.t_launch), float(r.t_encoded - r.t_done), float(t - r.t_encoded)};
    }
    bool push_token = false, last = false;
    {
      std::lock_guard<std::mutex> lk(mu);
      ++running;
      last = ++completed == total;
      if (r.code == kOk) {
        ++res.ok;
      } else {
        if (res.errors++ == 0) {
          res.first_error = r.message;
          res.first_error_code = r.code;
        }
      }
      if (open_loop) {
        if (i >= spec.warmup && i < spec.warmup + spec.count) {
          lat_sched[size_t(i)] = double(t - t_sched);
          stg_sched[size_t(i)] = sg;
        }
        if (completed == spec.warmup + spec.count) t_close = double(t);
      } else {
        // closed loop: the window is counted in completions, whatever their order
        if (completed == spec.warmup) t_open = double(t);
        if (completed > spec.warmup && completed <= spec.warmup + spec.count) {
          res.latency_us.push_back(double(t - t_sched));
          res.stages_us.push_back(sg);
        }
        if (completed == spec.warmup + spec.count) t_close = double(t);
        push_token = true;
      }
    }
    // test hook: hold the callback that counted the final completion here
    // (tests/test_live_server.py)
    if (spec.debug_done_delay_us > 0 && last)
      std::this_thread::sleep_for(std::chrono::microseconds(spec.debug_done_delay_us));
    if (push_token) {
      const int64_t k = next.fetch_add(1);
      if (k < total) work.push(k, 0);
    }
    std::lock_guard<std::mutex> lk(mu);
    if (--running == 0 && completed >= total) cv_all.notify_all();
  };

  std::vector<std::thread> subs;
  std::vector<int64_t> due;  // open loop: request i's send time
  const int T = std::max(1, spec.threads);
  const double wall0 = double(now_us());
  auto submit_one = [&](int64_t i, int64_t t_sched, int64_t t_pop) {
    const std::string& r = reqs[size_t(i % P)];
    const int64_t dl = spec.timeout_us > 0 ? t_sched + spec.timeout_us : 0;
    srv.submit(reinterpret_cast<const uint8_t*>(r.data()), r.size(), dl,
               [&on_done, i, t_sched, t_pop](Reply&& rep) { on_done(i, t_sched, t_pop, std::move(rep)); });
  };
  if (!open_loop) {
    for (int s = 0; s < T; ++s) {
      subs.emplace_back([&] {
        std::pair<int64_t, int64_t> w;
        while (work.pop(&w)) {
          const int64_t t_pop = now_us();
          submit_one(w.first, t_pop, t_pop);
        }
      });
    }
    if (spec.warmup == 0) t_open = double(now_us());
    for (int c = 0; c < C && c < total; ++c) work.push(next.fetch_add(1), 0);
  } else {
    // request i is due at t0 + i / qps (uniform) or at exponential gaps. No
    // shared queue and no schedule thread: each submitter claims the next
    // request (one atomic increment), waits until it is due and sends it, so
    // a submitter that stalls (preempted, a slow copy) holds up one request
    // while the others take the following ones. (One schedule thread pushing
    // every request through a condition variable fell behind at ~250 k
    // requests/s, and submitters that each owned every T-th request drained a
    // stall alone: both showed up as 10-50 ms latency tails at 75-90 % of
    // DeepFM's capacity, profiles/r06_latency_stages.md.)
    due.assign(static_cast<size_t>(total), 0);  // outlives this block: the submitters read it
    std::mt19937_64 rng(spec.seed);
    std::exponential_distribution<double> expo(spec.qps);
    const double t0 = double(now_us()) + 1000.0;
    double t_next = t0;
    for (int64_t i = 0; i < total; ++i) {
      due[size_t(i)] = int64_t(t_next);
      t_next += spec.poisson ? expo(rng) * 1e6 : 1e6 / spec.qps;
    }
    t_open = double(due[size_t(std::min<int64_t>(spec.warmup, total - 1))]);
    for (int s = 0; s < T; ++s) {
      subs.emplace_back([&] {
        for (;;) {
          const int64_t i = next.fetch_add(1);
          if (i >= total) break;
          const int64_t t_sched = due[size_t(i)];
          for (;;) {
            const int64_t now = now_us();
            if (now >= t_sched) break;
            const int64_t gap = t_sched - now;
            if (gap > 200) std::this_thread::sleep_for(std::chrono::microseconds(gap - 100));
            else std::this_thread::yield();
          }
          submit_one(i, t_sched, now_us());
        }
      });
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu);
    cv_all.wait(lk, [&] { return completed >= total && running == 0; });
  }
  work.close();
  for (auto& t : subs) t.join();
  res.submitted = total;
  res.wall_us = double(now_us()) - wall0;
  res.window_us = t_close - t_open;
  if (open_loop) {
    for (int64_t i = spec.warmup; i < spec.warmup + spec.count; ++i)
      if (lat_sched[size_t(i)] >= 0) {
        res.latency_us.push_back(lat_sched[size_t(i)]);
        res.stages_us.push_back(stg_sched[size_t(i)]);
      }
  }
  return res;
}

}  // namespace runtime
}  // namespace dtfs

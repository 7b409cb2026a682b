// Host-only stress driver of the native serving runtime for ThreadSanitizer
// (and ASan): LiveServer + load generator + step control, no Python, no GPU.
//
//   bash scripts/sanitize_native.sh   (SAN=thread builds and runs this too)
//
// The Python-hosted suites cannot run under TSan cleanly (the interpreter and
// torch are not instrumented), so this drives the same C++ objects the served
// path uses from C++ threads: submitters (run_load), the launcher, completer
// and watcher threads, and - in cluster mode - two ranks agreeing on every
// step through one shared-memory StepControl. The backend is a fake device:
// launch() records the step and fills the bucket's scores after a short
// "device time"; wait() honours the timeout. Scenarios: closed loop, open loop,
// close() while requests are queued, a broken cluster (mark_broken) with
// requests in flight, two ranks serving concurrently, and three ranks of a
// shared-arena scatter (runtime/shared_scatter.h) cycling the plan ring.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime/live_server.h"
#include "runtime/loadgen.h"
#include "runtime/shared_scatter.h"
#include "runtime/step_control.h"
#include "wire/tensor_codec.h"

using namespace dtfs;
using namespace dtfs::runtime;

namespace {

class FakeDevice : public StepBackend {
 public:
  FakeDevice(int slots, std::vector<int64_t> buckets, int64_t device_us)
      : buckets_(std::move(buckets)), device_us_(device_us), done_at_(size_t(slots), 0) {
    for (int s = 0; s < slots; ++s) {
      std::vector<std::vector<float>> per;
      for (int64_t b : buckets_) per.emplace_back(size_t(b), 0.f);
      scores_.push_back(std::move(per));
    }
  }
  int slots() const override { return int(scores_.size()); }
  const std::vector<int64_t>& buckets() const override { return buckets_; }
  void launch(int slot, int b, const uint8_t*, const ArenaBatch& batch) override {
    auto& s = scores_[size_t(slot)][size_t(b)];
    for (size_t i = 0; i < s.size(); ++i) s[i] = float(i % 97) / 97.f;
    (void)batch;
    std::lock_guard<std::mutex> lk(mu_);
    done_at_[size_t(slot)] = now() + device_us_;
    ++launched_;
  }
  bool wait(int slot, int64_t timeout_us, std::string* err) override {
    int64_t t;
    {
      std::lock_guard<std::mutex> lk(mu_);
      t = done_at_[size_t(slot)];
    }
    const int64_t dt = t - now();
    if (dt > timeout_us) {
      *err = "fake step timed out";
      return false;
    }
    if (dt > 0) std::this_thread::sleep_for(std::chrono::microseconds(dt));
    return true;
  }
  const float* scores(int slot, int b) const override { return scores_[size_t(slot)][size_t(b)].data(); }
  int64_t scores_len(int slot, int b) const override { return int64_t(scores_[size_t(slot)][size_t(b)].size()); }
  int64_t launched() const {
    std::lock_guard<std::mutex> lk(mu_);
    return launched_;
  }

 private:
  static int64_t now() {
    return std::chrono::duration_cast<std::chrono::microseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  std::vector<int64_t> buckets_;
  int64_t device_us_;
  mutable std::mutex mu_;
  std::vector<int64_t> done_at_;
  int64_t launched_ = 0;
  std::vector<std::vector<std::vector<float>>> scores_;
};

std::vector<std::string> make_requests(int n, int rows, int fields, bool raw) {
  std::vector<std::string> out;
  for (int r = 0; r < n; ++r) {
    std::vector<int64_t> ids(size_t(rows) * fields);
    std::vector<float> wts(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
      ids[i] = int64_t((i * 2654435761ull + r) % 100003);
      wts[i] = float((i + r) % 7) / 7.f;
    }
    wire::ModelSpecOut spec{"DCN", "serving_default", false, 0};
    std::vector<wire::TensorOut> in(2);
    in[0] = {"feat_ids", wire::DT_INT64, {rows, fields}, ids.data(), int64_t(ids.size()), raw};
    in[1] = {"feat_wts", wire::DT_FLOAT, {rows, fields}, wts.data(), int64_t(wts.size()), raw};
    out.push_back(wire::encode_predict_request(spec, in, {}));
  }
  return out;
}

struct Arenas {
  std::vector<std::unique_ptr<uint8_t[]>> mem;
  std::vector<std::pair<uint8_t*, int64_t>> list;
  Arenas(int n, int64_t bytes) {
    for (int i = 0; i < n; ++i) {
      mem.emplace_back(new uint8_t[size_t(bytes)]);
      std::memset(mem.back().get(), 0, size_t(bytes));
      list.emplace_back(mem.back().get(), bytes);
    }
  }
};

int fails = 0;
void check(bool ok, const char* what) {
  std::printf("%s %s\n", ok ? "ok  " : "FAIL", what);
  if (!ok) ++fails;
}

LiveConfig base_cfg() {
  LiveConfig c;
  c.fields = 43;
  c.max_batch_rows = 256;
  c.batch_timeout_us = 200;
  c.depth = 3;
  c.step_timeout_us = 2'000'000;
  return c;
}

void single_rank() {
  FakeDevice dev(3, {64, 256}, 150);
  Arenas ar(6, 4 << 20);
  LiveServer srv(&dev, base_cfg(), ar.list);
  const auto raw = make_requests(8, 40, 43, true), packed = make_requests(8, 33, 43, false);
  std::vector<std::string> mix(raw);
  mix.insert(mix.end(), packed.begin(), packed.end());
  LoadSpec closed;
  closed.warmup = 20, closed.count = 400, closed.concurrency = 24, closed.threads = 4, closed.timeout_us = 5'000'000;
  const LoadResult r = run_load(srv, mix, closed);
  check(r.errors == 0 && r.ok == r.submitted, "closed loop: every request answered OK");
  LoadSpec open;
  open.warmup = 10, open.count = 300, open.qps = 20000, open.poisson = true, open.threads = 3;
  open.debug_done_delay_us = 20'000;  // the final callback lingers: run_load must wait for it
  const LoadResult q = run_load(srv, mix, open);
  check(q.errors == 0 && q.wall_us >= 20'000, "open loop + lingering final callback");
  srv.close();
  check(srv.stats().completed >= r.ok + q.ok, "close() after load");
}

void close_under_load() {
  FakeDevice dev(2, {64, 256}, 300);
  Arenas ar(5, 4 << 20);
  auto srv = std::make_unique<LiveServer>(&dev, base_cfg(), ar.list);
  const auto reqs = make_requests(4, 50, 43, true);
  std::atomic<int> answered{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&] {
      for (int i = 0; i < 60; ++i)
        srv->submit(reinterpret_cast<const uint8_t*>(reqs[size_t(i) % reqs.size()].data()), reqs[0].size(), 0,
                    [&](Reply&&) { answered.fetch_add(1); });
    });
  std::this_thread::sleep_for(std::chrono::milliseconds(3));
  srv->close();  // racing the submitters: later submits are rejected, admitted ones finish
  for (auto& t : ts) t.join();
  srv.reset();
  check(answered.load() == 240, "close() racing submitters: every request answered exactly once");
}

void two_ranks(bool break_midway) {
  const std::string name = "/dtfs-stress-" + std::to_string(::getpid()) + (break_midway ? "-b" : "-a");
  StepControl c0(name, 2, 0, true);
  StepControl c1(name, 2, 1, false);
  c0.unlink();
  FakeDevice d0(3, {64, 256}, 120), d1(3, {64, 256}, 180);
  Arenas a0(6, 4 << 20), a1(6, 4 << 20);
  LiveConfig cfg = base_cfg();
  cfg.peer_timeout_us = 2'000'000;
  cfg.heartbeat_us = 2'000;
  LiveServer s0(&d0, cfg, a0.list, &c0), s1(&d1, cfg, a1.list, &c1);
  const auto reqs = make_requests(6, 37, 43, true);
  LoadSpec ls;
  ls.warmup = 10, ls.count = break_midway ? 2000 : 200, ls.concurrency = 12, ls.threads = 3,
  ls.timeout_us = 5'000'000;
  LoadResult r0, r1;
  std::thread t0([&] { r0 = run_load(s0, reqs, ls); });
  std::thread t1([&] { r1 = run_load(s1, reqs, ls); });
  if (break_midway) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    c1.mark_broken(1);  // rank 1 gives up: both servers fail what is in flight, then reject
  }
  t0.join();
  t1.join();
  if (break_midway) {
    check(s0.broken() && s1.broken() && r0.errors > 0 && r0.ok + r0.errors == r0.submitted,
          "two ranks, cluster broken mid-load: every request answered, servers broken");
  } else {
    check(r0.errors == 0 && r1.errors == 0, "two ranks: every request answered OK");
    check(d0.launched() == d1.launched(), "two ranks: both ran the same steps");
  }
  // a closing rank keeps joining its peers' steps until every rank closes:
  // the ranks close concurrently, as separate processes do
  std::thread c([&] { s1.close(); });
  s0.close();
  c.join();
}

// Three ranks on one shared-scatter segment, one thread each: rank 0 builds a
// batch of a varying size in one of two shared arenas and publishes the plan;
// every rank copies its share (memcpy standing in for the DMA), checks it
// against the rows' own bytes, and marks the step done; rank 0 reuses an arena
// only after every rank finished the step that read it.
void shared_scatter_ring() {
  const std::string name = "/dtfs-stress-sct-" + std::to_string(getpid());
  const int W = 3, F = 43, B = 128, steps = 400;
  const int64_t cap = 8 << 20;
  SharedScatter s0(name, W, 0, true, F, 2, cap, 2, int64_t(W) * B);
  SharedScatter s1(name, W, 1, false), s2(name, W, 2, false);
  s0.unlink();
  const auto reqs = make_requests(12, 29, F, true);
  std::atomic<int> bad{0};
  auto take = [&](SharedScatter& s, uint64_t k, std::vector<uint8_t>& dst) {
    RankShare mine;
    int ai = -1;
    if (!s.wait_plan(k, 5'000'000, &mine, &ai)) {
      ++bad;
      return;
    }
    uint8_t hdr[64];
    const uint8_t* src = s.arena(ai);
    for (const auto& c : share_copies(src, mine, hdr)) std::memcpy(dst.data() + c.dst_off, c.src, size_t(c.n));
    int64_t rows, rt;
    std::memcpy(&rows, dst.data() + 8, 8);
    std::memcpy(&rt, src + 16, 8);
    if (rows != mine.rows) ++bad;
    // every row's table entry arrived at the table's start, and its ids match the source batch
    for (int64_t i = 0; i < mine.rows; ++i) {
      int32_t e[2], f[2];
      std::memcpy(e, dst.data() + kArenaPayloadOff + rt + 8 * i, 8);
      std::memcpy(f, src + kArenaPayloadOff + rt + 8 * (mine.row0 + i), 8);
      if (e[0] != f[0] || e[1] != f[1] ||
          std::memcmp(dst.data() + kArenaPayloadOff + (e[0] & 0x7fffffff), src + kArenaPayloadOff + (e[0] & 0x7fffffff),
                      8 * F) != 0)
        ++bad;
    }
    s.mark_done(k);
  };
  auto follower = [&](SharedScatter* s) {
    std::vector<uint8_t> dst(static_cast<size_t>(cap));
    for (int k = 0; k < steps; ++k) take(*s, s->begin_step(), dst);
  };
  std::thread t1(follower, &s1), t2(follower, &s2);
  std::vector<uint8_t> dst0(static_cast<size_t>(cap));
  for (int k = 0; k < steps; ++k) {
    const int ai = k % 2, n = 1 + k % 12;  // 29 .. 348 rows: some ranks get nothing
    std::vector<std::pair<const char*, size_t>> rq;
    for (int i = 0; i < n; ++i) rq.emplace_back(reqs[size_t(i)].data(), reqs[size_t(i)].size());
    uint8_t* a = s0.arena(ai);
    const auto spans = arena_place(a, cap, rq, 0);
    arena_build(a, cap, spans, "feat_ids", "feat_wts", F, int64_t(W) * B, 0);
    const uint64_t kk = s0.begin_step();
    s0.publish_plan(kk, ai, B);
    take(s0, kk, dst0);
    std::string err;
    if (!s0.wait_done(kk, 5'000'000, &err)) {
      ++bad;
      break;
    }
  }
  t1.join();
  t2.join();
  check(bad.load() == 0, "shared scatter: 3 ranks, every share copied and checked, plan ring reused");
}

}  // namespace

int main() {
  single_rank();
  close_under_load();
  two_ranks(false);
  two_ranks(true);
  shared_scatter_ring();
  std::printf("%s\n", fails ? "live_stress: FAILED" : "live_stress: all ok");
  return fails ? 1 : 0;
}

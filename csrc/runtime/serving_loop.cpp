#include "serving_loop.h"

#include <chrono>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <thread>

#include "../wire/tensor_codec.h"
#include "trace.h"

namespace dtfs {
namespace runtime {

namespace {
double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

ServingLoop::ServingLoop(StepRunner* runner, LoopConfig cfg, std::vector<LoopSlot> slots)
    : runner_(runner), cfg_(std::move(cfg)), slots_(std::move(slots)) {
  if (!runner_) throw std::invalid_argument("null StepRunner");
  if (cfg_.depth < 1) throw std::invalid_argument("depth must be >= 1");
  if (int(slots_.size()) < cfg_.depth + 1) throw std::invalid_argument("need slots >= depth + 1");
  if (int(slots_.size()) > runner_->slots()) throw std::invalid_argument("more loop slots than runner slots");
  for (const auto& s : slots_) {
    if (s.program ? !s.prog.h2d_dst
        : s.fanout ? (!(s.fan.forward || s.fan.forward_seq) || !s.fan.cin || !s.fan.cout)
                   : (!(s.graph || s.seq) || !s.h2d_dst))
      throw std::invalid_argument("incomplete loop slot");
    if (!s.h_out) throw std::invalid_argument("loop slot without host scores");
  }
}

void ServingLoop::add_input(uint8_t* arena, int64_t capacity, std::vector<Span> spans) {
  if (!arena || capacity <= kArenaPayloadOff) throw std::invalid_argument("bad arena");
  inputs_.push_back(Input{arena, capacity, std::move(spans)});
}

LoopStats ServingLoop::run(int64_t n, bool record) {
  if (inputs_.empty()) throw std::invalid_argument("no inputs registered");
  const int S = int(slots_.size());
  const int D = cfg_.depth;
  const int64_t P = int64_t(inputs_.size());
  if (P < D) throw std::invalid_argument("need at least `depth` inputs (an arena is reused only after its step ended)");
  LoopStats st;
  if (n <= 0) return st;

  std::vector<ArenaBatch> parsed(static_cast<size_t>(n));
  std::vector<double> t_start(size_t(n), 0.0), t_done(size_t(n), 0.0), sums(record ? size_t(n) : 0, 0.0);
  std::vector<char> parse_done(size_t(n), 0), finished(size_t(n), 0), encoded(size_t(n), 0);
  int64_t next_launch = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::exception_ptr err;
  bool abort = false;
  double parse_us = 0, encode_us = 0;
  int64_t resp_bytes = 0, n_req = 0, n_rows = 0, n_err = 0;

  wire::ModelSpecOut spec;
  spec.name = cfg_.model_name;
  spec.signature_name = cfg_.signature_name;
  spec.has_version = cfg_.version >= 0;
  spec.version = cfg_.version;

  auto fail = [&](std::exception_ptr e) {
    std::lock_guard<std::mutex> lk(mu);
    if (!err) err = e;
    abort = true;
    cv.notify_all();
  };

  std::thread parser([&] {
    try {
      for (int64_t k = 0; k < n; ++k) {
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return abort || (k < next_launch + D && (k < P || finished[size_t(k - P)])); });
          if (abort) return;
        }
        const Input& in = inputs_[size_t(k % P)];
        const double t0 = now_us();
        trace::Range tr("parse");
        ArenaBatch b = arena_build(in.arena, in.capacity, in.spans, cfg_.ids_key, cfg_.wts_key, cfg_.fields,
                                   cfg_.max_rows, cfg_.varint_chunks);
        const double t1 = now_us();
        std::lock_guard<std::mutex> lk(mu);
        parsed[size_t(k)] = std::move(b);
        t_start[size_t(k)] = t0;
        parse_us += t1 - t0;
        parse_done[size_t(k)] = 1;
        cv.notify_all();
      }
    } catch (...) {
      fail(std::current_exception());
    }
  });

  std::thread encoder([&] {
    try {
      for (int64_t j = 0; j < n; ++j) {
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return abort || finished[size_t(j)]; });
          if (abort) return;
        }
        const double t0 = now_us();
        trace::Range tr("encode");
        const ArenaBatch& b = parsed[size_t(j)];
        const LoopSlot& s = slots_[size_t(j % S)];
        int64_t bytes = 0, req = 0, rows = 0, errs = 0;
        double sum = 0;
        for (size_t i = 0; i < b.rows.size(); ++i) {
          if (!b.errors[i].empty() || b.offsets[i] + b.rows[i] > s.h_out_len) {
            ++errs;
            continue;
          }
          if (record)  // what the host actually read: checks the step-done signal's visibility
            for (int64_t r = 0; r < b.rows[i]; ++r) sum += double(s.h_out[b.offsets[i] + r]);
          wire::TensorOut t;
          t.key = cfg_.output_key;
          t.dtype = wire::DT_FLOAT;
          t.shape = {b.rows[i]};
          t.data = s.h_out + b.offsets[i];
          t.n = b.rows[i];
          t.raw = false;
          bytes += int64_t(wire::encode_predict_response(spec, {t}).size());
          ++req;
          rows += b.rows[i];
        }
        const double t1 = now_us();
        std::lock_guard<std::mutex> lk(mu);
        if (record) sums[size_t(j)] = sum;
        encode_us += t1 - t0;
        resp_bytes += bytes;
        n_req += req;
        n_rows += rows;
        n_err += errs;
        encoded[size_t(j)] = 1;
        cv.notify_all();
      }
    } catch (...) {
      fail(std::current_exception());
    }
  });

  double launch_us = 0, wait_us = 0;
  const bool s_fanout_any = slots_[0].fanout;
  const double wall0 = now_us();
  auto finish = [&](int64_t j) {
    const double t0 = now_us();
    trace::Range tr("gpu_wait");
    runner_->wait(int(j % S));
    const double t1 = now_us();
    wait_us += t1 - t0;
    std::lock_guard<std::mutex> lk(mu);
    t_done[size_t(j)] = t1;
    finished[size_t(j)] = 1;
    cv.notify_all();
  };
  try {
    for (int64_t k = 0; k < n; ++k) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return abort || (parse_done[size_t(k)] && (k < S || encoded[size_t(k - S)])); });
        if (abort) break;
      }
      const double t0 = now_us();
      trace::Range tr(s_fanout_any ? "launch_fanout" : "launch");
      const Input& in = inputs_[size_t(k % P)];
      const ArenaBatch& b = parsed[size_t(k)];
      const int slot = int(k % S);
      const LoopSlot& s = slots_[size_t(slot)];
      const int64_t nbytes = b.n_valid > 0 ? b.used_bytes : 0;
      if (s.program) {
        runner_->launch_program(slot, s.prog, in.arena, nbytes, b.n_gpu_varint == 0);
      } else if (s.fanout) {
        FanoutStep f = s.fan;
        f.h2d_src = in.arena;
        f.h2d_bytes = nbytes;
        runner_->launch_fanout(slot, f);
      } else {
        if (s.seq) runner_->launch_seq(slot, s.h2d_dst, in.arena, nbytes, s.seq, b.n_gpu_varint == 0);
        else runner_->launch(slot, s.h2d_dst, in.arena, nbytes, s.graph);
      }
      launch_us += now_us() - t0;
      {
        std::lock_guard<std::mutex> lk(mu);
        next_launch = k + 1;
        cv.notify_all();
      }
      if (k - D + 1 >= 0) finish(k - D + 1);
    }
    if (!abort)
      for (int64_t j = std::max<int64_t>(0, n - D + 1); j < n; ++j) finish(j);
  } catch (...) {
    fail(std::current_exception());
  }
  parser.join();
  encoder.join();
  if (err) std::rethrow_exception(err);
  st.wall_us = now_us() - wall0;
  st.steps = n;
  st.requests = n_req;
  st.rows = n_rows;
  st.errors = n_err;
  st.response_bytes = resp_bytes;
  st.parse_us = parse_us;
  st.encode_us = encode_us;
  st.launch_us = launch_us;
  st.wait_us = wait_us;
  if (record) {
    st.latency_us.resize(size_t(n));
    for (int64_t k = 0; k < n; ++k) st.latency_us[size_t(k)] = t_done[size_t(k)] - t_start[size_t(k)];
    st.score_sum = std::move(sums);
  }
  return st;
}

}  // namespace runtime
}  // namespace dtfs

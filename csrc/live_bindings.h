// Python surface of runtime::LiveServer, shared by _native (CPU backend) and
// _hip (GPU backend). Each module registers its own LiveServer class around a
// holder type H with members `srv` (std::unique_ptr<LiveServer>) and `keep`
// (Python objects whose memory the server points into).
#pragma once

#include <torch/extension.h>

#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include <condition_variable>
#include <deque>
#include <thread>

#include "net/h2_server.h"
#include "runtime/batcher.h"
#include "runtime/numa.h"
#include "runtime/live_server.h"
#include "runtime/loadgen.h"
#include "runtime/shared_scatter.h"
#include "runtime/step_control.h"

namespace dtfs_live {

namespace py = pybind11;
using dtfs::runtime::LiveConfig;
using dtfs::runtime::LiveServer;
using dtfs::runtime::Reply;
using dtfs::runtime::StepControl;

// StepControl (runtime/step_control.h) of this module; module-local, so the
// CPU (_native) and GPU (_hip) modules each own one binding of the type.
inline void def_step_control(py::module& m) {
  py::class_<StepControl>(m, "StepControl", py::module_local(),
                          "Shared-memory step agreement of a multi-rank live server (one node)")
      .def(py::init<std::string, int, int, bool>(), py::arg("name"), py::arg("world"), py::arg("rank"),
           py::arg("create"))
      .def_property_readonly("world", &StepControl::world)
      .def_property_readonly("rank", &StepControl::rank)
      .def_property_readonly("name", &StepControl::name)
      .def_property_readonly("proposed", &StepControl::proposed)
      .def("propose", &StepControl::propose, py::arg("step"))
      .def("post", &StepControl::post, py::arg("step"), py::arg("bucket"))
      .def(
          "gather",
          [](StepControl& c, uint64_t k, double timeout_s) {
            std::string err;
            int b;
            {
              py::gil_scoped_release nogil;
              b = c.gather(k, int64_t(timeout_s * 1e6), &err);
            }
            return py::make_tuple(b, err);
          },
          py::arg("step"), py::arg("timeout_s"))
      .def("heartbeat", &StepControl::heartbeat)
      .def(
          "silent_peer", [](const StepControl& c, double timeout_s) { return c.silent_peer(int64_t(timeout_s * 1e6)); },
          py::arg("timeout_s"))
      .def(
          "heartbeat_age", [](const StepControl& c, int r) { return double(c.heartbeat_age_us(r)) * 1e-6; },
          py::arg("rank"), "seconds since the rank's last heartbeat (huge once its process exited)")
      .def("process_gone", &StepControl::process_gone, py::arg("rank"), "the rank's process no longer exists")
      .def("set_closing", &StepControl::set_closing, py::arg("closing"))
      .def_property_readonly("all_closing", &StepControl::all_closing)
      .def("request_stop", &StepControl::request_stop)
      .def_property_readonly("stop_requested", &StepControl::stop_requested)
      .def("mark_broken", &StepControl::mark_broken, py::arg("by_rank"))
      .def_property_readonly("broken_by", &StepControl::broken_by)
      .def_property_readonly("epoch", &StepControl::epoch)
      .def("bump_epoch", &StepControl::bump_epoch)
      .def(
          "wait_event",
          [](StepControl& c, double timeout_s) {
            // block until a stop request, a broken cluster, an epoch change or
            // the timeout; heartbeats while waiting (a follower's main thread)
            py::gil_scoped_release nogil;
            const int64_t end = dtfs::runtime::now_us() + int64_t(timeout_s * 1e6);
            const uint32_t ep = c.epoch();
            for (;;) {
              const uint32_t seen = c.bell();
              c.heartbeat();
              if (c.stop_requested() || c.broken_by() >= 0 || c.epoch() != ep) return true;
              const int64_t left = end - dtfs::runtime::now_us();
              if (left <= 0) return false;
              c.wait_bell(seen, std::min<int64_t>(left, 20000));
            }
          },
          py::arg("timeout_s"))
      .def("unlink", &StepControl::unlink);
}

// SharedScatter (runtime/shared_scatter.h) of this module (module-local like
// StepControl). Host-side operations only; the GPU module adds registration
// and the device launch (bindings_hip.cpp).
using dtfs::runtime::SharedScatter;
using ScatterClass = py::class_<SharedScatter, std::shared_ptr<SharedScatter>>;

inline ScatterClass def_shared_scatter(py::module& m) {
  ScatterClass c(m, "SharedScatter", py::module_local(),
                 "Scatter fan-out through rank 0's shared request arenas (one node; runtime/shared_scatter.h)");
  c.def(py::init<std::string, int, int, bool, int64_t, int, int64_t, int, int64_t, int, std::vector<int>, int64_t>(),
        py::arg("name"), py::arg("world"), py::arg("rank"), py::arg("create"), py::arg("fields") = 0,
        py::arg("n_arenas") = 0, py::arg("arena_cap") = 0, py::arg("slots") = 0, py::arg("out_floats") = 0,
        py::arg("node") = -1, py::arg("rank_nodes") = std::vector<int>(), py::arg("expected_payload") = 0)
      .def(
          "placement",
          [](const SharedScatter& s) {
            py::list l;
            for (const auto& sl : s.placement())
              l.append(py::dict(py::arg("lo") = sl.lo, py::arg("hi") = sl.hi, py::arg("node") = sl.node,
                                py::arg("rank") = sl.rank, py::arg("bound") = sl.bound));
            return l;
          },
          "per-rank NUMA slices of the arenas placed at creation: [{lo, hi, node, rank, bound}] (segment offsets)")
      .def(
          "page_node",
          [](const SharedScatter& s, int64_t off) {
            TORCH_CHECK(off >= 0 && size_t(off) < s.bytes(), "offset outside the segment");
            return dtfs::runtime::page_numa_node(static_cast<const uint8_t*>(s.base()) + off);
          },
          py::arg("offset"), "NUMA node of the page at a segment offset (-1 untouched / unknown)")
      .def_property_readonly("world", &SharedScatter::world)
      .def_property_readonly("rank", &SharedScatter::rank)
      .def_property_readonly("n_arenas", &SharedScatter::n_arenas)
      .def_property_readonly("slots", &SharedScatter::slots)
      .def_property_readonly("arena_cap", &SharedScatter::arena_cap)
      .def_property_readonly("out_floats", &SharedScatter::out_floats)
      .def_property_readonly("h2d_bytes", &SharedScatter::h2d_bytes)
      .def_property_readonly("h2d_steps", &SharedScatter::h2d_steps)
      .def_property_readonly("all_attached", &SharedScatter::all_attached)
      .def("unlink", &SharedScatter::unlink)
      // views into the mapping: valid while this object lives (the engine keeps it)
      .def(
          "arena",
          [](SharedScatter& s, int i) {
            return torch::from_blob(s.arena(i), {s.arena_cap()}, torch::TensorOptions().dtype(torch::kUInt8));
          },
          py::arg("index"))
      .def(
          "out",
          [](SharedScatter& s, int slot) {
            return torch::from_blob(s.out(slot), {s.out_floats()}, torch::TensorOptions().dtype(torch::kFloat32));
          },
          py::arg("slot"))
      .def(
          "arena_index",
          [](SharedScatter& s, torch::Tensor t) { return s.arena_index(static_cast<const uint8_t*>(t.data_ptr())); },
          py::arg("arena"))
      .def("begin_step", &SharedScatter::begin_step)
      .def("publish_plan", &SharedScatter::publish_plan, py::arg("step"), py::arg("arena_index"),
           py::arg("rows_per_rank"))
      .def(
          "take_share",
          [](SharedScatter& s, uint64_t k, torch::Tensor dst, double timeout_s) {
            // host path (CPU backend): wait for step k's plan and copy this
            // rank's share into dst (an arena of the same layout) with memcpy
            TORCH_CHECK(dst.device().is_cpu() && dst.is_contiguous() && dst.scalar_type() == torch::kUInt8 &&
                            dst.numel() >= s.arena_cap(),
                        "dst must be a contiguous CPU uint8 arena of the segment's capacity");
            dtfs::runtime::RankShare mine;
            int ai = -1;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.wait_plan(k, int64_t(timeout_s * 1e6), &mine, &ai);
            }
            TORCH_CHECK(ok, "shared scatter: no plan for step ", k, " from rank 0");
            uint8_t hdr[64];
            const auto copies = dtfs::runtime::share_copies(s.arena(ai), mine, hdr);
            uint8_t* d = dst.data_ptr<uint8_t>();
            int64_t n = 0;
            for (const auto& cp : copies) {
              std::memcpy(d + cp.dst_off, cp.src, size_t(cp.n));
              n += cp.n;
            }
            s.add_h2d(n);
            return py::make_tuple(mine.row0, mine.rows, n);
          },
          py::arg("step"), py::arg("dst"), py::arg("timeout_s") = 10.0)
      .def("mark_done", &SharedScatter::mark_done, py::arg("step"))
      .def("compact_scores", &SharedScatter::compact_scores, py::arg("step"), py::arg("slot"))
      .def(
          "wait_done",
          [](const SharedScatter& s, uint64_t k, double timeout_s) {
            std::string err;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.wait_done(k, int64_t(timeout_s * 1e6), &err);
            }
            return py::make_tuple(ok, err);
          },
          py::arg("step"), py::arg("timeout_s"))
      .def_static(
          "shares",
          [](torch::Tensor arena, int64_t fields, int world, int64_t rows_per_rank) {
            // plan of a built arena, for tests: [(row0, rows, [(lo, hi), ...]), ...]
            TORCH_CHECK(arena.device().is_cpu() && arena.is_contiguous(), "arena must be a contiguous CPU tensor");
            std::vector<dtfs::runtime::RankShare> sh(static_cast<size_t>(world));
            dtfs::runtime::compute_shares(arena.data_ptr<uint8_t>(), arena.numel(), fields, world, rows_per_rank,
                                          sh.data());
            py::list out;
            for (const auto& r : sh) {
              py::list rg;
              for (int i = 0; i < r.n_ranges; ++i) rg.append(py::make_tuple(r.r[i].lo, r.r[i].hi));
              out.append(py::make_tuple(r.row0, r.rows, rg));
            }
            return out;
          },
          py::arg("arena"), py::arg("fields"), py::arg("world"), py::arg("rows_per_rank"));
  return c;
}

inline SharedScatter* scatter_from(const py::object& o, std::vector<py::object>* keep) {
  if (o.is_none()) return nullptr;
  keep->push_back(o);
  return &o.cast<SharedScatter&>();
}

inline StepControl* control_from(const py::object& o, std::vector<py::object>* keep) {
  if (o.is_none()) return nullptr;
  keep->push_back(o);
  return &o.cast<StepControl&>();
}

inline LiveConfig live_config_from(const py::dict& d) {
  LiveConfig c;
  auto get = [&](const char* k) { return d.contains(k) && !d[k].is_none(); };
  if (get("fields")) c.fields = d["fields"].cast<int64_t>();
  if (get("ids_key")) c.ids_key = d["ids_key"].cast<std::string>();
  if (get("wts_key")) c.wts_key = d["wts_key"].cast<std::string>();
  if (get("model_name")) c.model_name = d["model_name"].cast<std::string>();
  if (get("signature_name")) c.signature_name = d["signature_name"].cast<std::string>();
  if (get("output_key")) c.output_key = d["output_key"].cast<std::string>();
  if (get("caller_outputs")) c.caller_outputs = d["caller_outputs"].cast<std::vector<std::string>>();
  if (get("version")) c.version = d["version"].cast<int64_t>();
  if (get("max_batch_rows")) c.max_batch_rows = d["max_batch_rows"].cast<int64_t>();
  if (get("batch_timeout_us")) c.batch_timeout_us = d["batch_timeout_us"].cast<int64_t>();
  if (get("depth")) c.depth = d["depth"].cast<int>();
  if (get("varint_chunks")) c.varint_chunks = d["varint_chunks"].cast<int64_t>();
  if (get("max_pending")) c.max_pending = d["max_pending"].cast<int64_t>();
  if (get("eager_when_idle")) c.eager_when_idle = d["eager_when_idle"].cast<bool>();
  if (get("peer_timeout_us")) c.peer_timeout_us = d["peer_timeout_us"].cast<int64_t>();
  if (get("heartbeat_us")) c.heartbeat_us = d["heartbeat_us"].cast<int64_t>();
  if (get("step_timeout_us")) c.step_timeout_us = d["step_timeout_us"].cast<int64_t>();
  if (get("start_paused")) c.start_paused = d["start_paused"].cast<bool>();
  if (get("liveness_only")) c.liveness_only = d["liveness_only"].cast<bool>();
  if (get("narrow_modulo")) c.narrow_modulo = d["narrow_modulo"].cast<int64_t>();
  if (get("narrow_wts_cols")) c.narrow_wts_cols = d["narrow_wts_cols"].cast<int64_t>();
  return c;
}

// Host arenas: contiguous uint8 CPU tensors (pinned for a GPU backend).
inline std::vector<std::pair<uint8_t*, int64_t>> arenas_from(const py::list& arenas, bool need_pinned,
                                                             std::vector<py::object>* keep) {
  std::vector<std::pair<uint8_t*, int64_t>> out;
  for (auto a : arenas) {
    torch::Tensor t = a.cast<torch::Tensor>();
    TORCH_CHECK(t.device().is_cpu() && t.is_contiguous() && t.scalar_type() == torch::kUInt8,
                "arenas must be contiguous CPU uint8 tensors");
    TORCH_CHECK(!need_pinned || t.is_pinned(), "a GPU live server needs pinned arenas");
    keep->push_back(py::reinterpret_borrow<py::object>(a));
    out.emplace_back(t.data_ptr<uint8_t>(), t.numel());
  }
  return out;
}

inline int64_t deadline_from(double timeout_s) {
  return timeout_s > 0 ? dtfs::runtime::now_us() + int64_t(timeout_s * 1e6) : 0;
}

inline std::pair<const uint8_t*, size_t> bytes_view(const py::bytes& b) {
  char* p;
  Py_ssize_t n;
  if (PyBytes_AsStringAndSize(b.ptr(), &p, &n) != 0) throw py::error_already_set();
  return {reinterpret_cast<const uint8_t*>(p), size_t(n)};
}

template <class H>
void def_live_methods(py::class_<H>& c) {
  c.def(
       "predict",
       [](H& h, py::bytes data, double timeout_s) {
         auto v = bytes_view(data);
         Reply r;
         {
           py::gil_scoped_release nogil;
           r = h.srv->predict(v.first, v.second, deadline_from(timeout_s));
         }
         return py::make_tuple(r.code, r.message, py::bytes(r.response));
       },
       py::arg("request"), py::arg("timeout_s") = 0.0,
       "Serve one serialized PredictRequest; returns (code, message, response bytes). code 0 = OK, otherwise a "
       "gRPC status code (1000: more rows than one batch, split and resubmit).")
      .def(
          "submit",
          [](H& h, py::bytes data, double timeout_s, py::function cb) {
            auto v = bytes_view(data);
            // the callback object is released with the GIL held, wherever the
            // last reference goes away
            auto fn = std::shared_ptr<py::function>(new py::function(cb), [](py::function* f) {
              py::gil_scoped_acquire g;
              delete f;
            });
            const int64_t dl = deadline_from(timeout_s);
            py::gil_scoped_release nogil;
            h.srv->submit(v.first, v.second, dl, [fn](Reply&& r) {
              py::gil_scoped_acquire g;
              try {
                (*fn)(r.code, r.message, py::bytes(r.response));
              } catch (py::error_already_set& e) {
                e.discard_as_unraisable("LiveServer completion callback");
              }
            });
          },
          py::arg("request"), py::arg("timeout_s"), py::arg("callback"),
          "Asynchronous submit: callback(code, message, response) runs on the server's completion thread.")
      .def(
          "run_load",
          [](H& h, const std::vector<std::string>& requests, py::dict spec) {
            dtfs::runtime::LoadSpec s;
            auto get = [&](const char* k) { return spec.contains(k) && !spec[k].is_none(); };
            if (get("warmup")) s.warmup = spec["warmup"].cast<int64_t>();
            if (get("count")) s.count = spec["count"].cast<int64_t>();
            if (get("tail")) s.tail = spec["tail"].cast<int64_t>();
            if (get("concurrency")) s.concurrency = spec["concurrency"].cast<int>();
            if (get("qps")) s.qps = spec["qps"].cast<double>();
            if (get("poisson")) s.poisson = spec["poisson"].cast<bool>();
            if (get("threads")) s.threads = spec["threads"].cast<int>();
            if (get("timeout_us")) s.timeout_us = spec["timeout_us"].cast<int64_t>();
            if (get("seed")) s.seed = spec["seed"].cast<uint64_t>();
            if (get("debug_done_delay_us")) s.debug_done_delay_us = spec["debug_done_delay_us"].cast<int64_t>();
            dtfs::runtime::LoadResult r;
            {
              py::gil_scoped_release nogil;
              r = dtfs::runtime::run_load(*h.srv, requests, s);
            }
            py::dict o;
            o["latency_us"] = r.latency_us;
            // [n, 6] float32: sched_lag, admit, batch, step, encode, deliver (loadgen.h Stages)
            py::array_t<float> stg({py::ssize_t(r.stages_us.size()), py::ssize_t(dtfs::runtime::kStages)});
            if (!r.stages_us.empty())
              std::memcpy(stg.mutable_data(), r.stages_us.data(), r.stages_us.size() * sizeof(dtfs::runtime::Stages));
            o["stages_us"] = stg;
            o["submitted"] = r.submitted;
            o["ok"] = r.ok;
            o["errors"] = r.errors;
            o["window_us"] = r.window_us;
            o["wall_us"] = r.wall_us;
            o["first_error"] = r.first_error;
            o["first_error_code"] = r.first_error_code;
            return o;
          },
          py::arg("requests"), py::arg("spec"),
          "Native load generator over submit(): closed loop (concurrency) or open loop (qps).")
      .def(
          "stats",
          [](H& h) {
            auto s = h.srv->stats();
            py::dict o;
            o["submitted"] = s.submitted;
            o["rejected"] = s.rejected;
            o["completed"] = s.completed;
            o["failed"] = s.failed;
            o["expired"] = s.expired;
            o["steps"] = s.steps;
            o["rows"] = s.rows;
            o["padded_rows"] = s.padded_rows;
            o["empty_steps"] = s.empty_steps;
            o["full_steps"] = s.full_steps;
            o["timeout_steps"] = s.timeout_steps;
            o["eager_steps"] = s.eager_steps;
            o["blocked_submits"] = s.blocked_submits;
            o["narrowed"] = s.narrowed;
            o["narrowed_wts_bf16"] = s.narrowed_wts_bf16;
            o["narrowed_wts_implicit"] = s.narrowed_wts_implicit;
            o["proposed_steps"] = s.proposed_steps;
            o["joined_steps"] = s.joined_steps;
            o["copy_us"] = s.copy_us;
            o["build_us"] = s.build_us;
            o["launch_us"] = s.launch_us;
            o["wait_us"] = s.wait_us;
            o["encode_us"] = s.encode_us;
            o["broken"] = s.broken;
            o["error"] = s.error;
            return o;
          })
      .def("resume", [](H& h) { h.srv->resume(); })
      .def("close", [](H& h) {
        py::gil_scoped_release nogil;
        h.srv->close();
      })
      .def_property_readonly("broken", [](H& h) { return h.srv->broken(); })
      .def_property_readonly("max_rows", [](H& h) { return h.srv->max_rows(); });
}

// ---- native gRPC front door (csrc/net/h2_server.h) -------------------------
// Predict goes straight into this module's LiveServer::submit on the event
// loop thread; everything else (the other four PredictionService RPCs, and
// Predicts the fast path hands back: ranked outputs, more rows than a batch)
// goes to a Python handler on a few worker threads.
class FallbackPool {
 public:
  FallbackPool(py::function fn, int threads)
      : fn_(new py::function(std::move(fn)), [](py::function* f) {
          py::gil_scoped_acquire g;
          delete f;
        }) {
    for (int i = 0; i < std::max(1, threads); ++i) ts_.emplace_back([this] { work(); });
  }
  ~FallbackPool() { stop(); }
  void push(dtfs::net::GrpcCall&& c, dtfs::net::Responder r) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!stop_) {
        q_.emplace_back(std::move(c), std::move(r));
        cv_.notify_one();
        return;
      }
    }
    r.reply(14, "server is shutting down", "");
  }
  void stop() {  // call without the GIL
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : ts_)
      if (t.joinable()) t.join();
    ts_.clear();
  }

 private:
  void work() {
    for (;;) {
      std::pair<dtfs::net::GrpcCall, dtfs::net::Responder> item;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        item = std::move(q_.front());
        q_.pop_front();
      }
      const auto& c = item.first;
      const double timeout_s =
          c.deadline_us > 0 ? std::max(1e-3, double(c.deadline_us - dtfs::runtime::now_us()) * 1e-6) : 0.0;
      int status = 13;
      std::string msg, body;
      {
        py::gil_scoped_acquire g;
        try {
          py::tuple t = (*fn_)(c.path, py::bytes(c.message), timeout_s);
          status = t[0].cast<int>();
          msg = t[1].cast<std::string>();
          body = t[2].cast<std::string>();
        } catch (py::error_already_set& e) {
          msg = e.what();
        } catch (const std::exception& e) {
          msg = e.what();
        }
      }
      item.second.reply(status, std::move(msg), std::move(body));
    }
  }
  std::shared_ptr<py::function> fn_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<dtfs::net::GrpcCall, dtfs::net::Responder>> q_;
  bool stop_ = false;
  std::vector<std::thread> ts_;
};

// Predicts the event loop could not admit without blocking (every arena queued
// or in flight: LiveServer::try_submit false) wait for a batch slot here, on a
// few native threads, so the loop keeps serving PINGs, WINDOW_UPDATEs and the
// replies of other connections. Bounded: past kMaxQueued the call is answered
// RESOURCE_EXHAUSTED at once.
class SubmitPool {
 public:
  static constexpr size_t kMaxQueued = 4096;
  explicit SubmitPool(int threads) {
    for (int i = 0; i < std::max(1, threads); ++i) ts_.emplace_back([this] { work(); });
  }
  ~SubmitPool() { stop(); }
  bool push(std::function<void()> task) {
    std::lock_guard<std::mutex> lk(mu_);
    if (stop_ || q_.size() >= kMaxQueued) return false;
    q_.push_back(std::move(task));
    ++handed_;
    cv_.notify_one();
    return true;
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : ts_)
      if (t.joinable()) t.join();
    ts_.clear();
  }
  int64_t handed() const {
    std::lock_guard<std::mutex> lk(mu_);
    return handed_;
  }

 private:
  void work() {
    for (;;) {
      std::function<void()> task;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stopping and drained: queued submits still run first
        task = std::move(q_.front());
        q_.pop_front();
      }
      task();
    }
  }
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  int64_t handed_ = 0;
  std::vector<std::thread> ts_;
};

struct GrpcFront {
  py::object live;  // the LiveServer holder: outlives the front door
  std::shared_ptr<FallbackPool> fb;
  std::shared_ptr<SubmitPool> sp;
  std::unique_ptr<dtfs::net::H2GrpcServer> h2;
  void stop() {
    py::gil_scoped_release nogil;
    if (h2) h2->stop();
    if (sp) sp->stop();
    if (fb) fb->stop();
  }
  ~GrpcFront() {
    try {
      stop();
    } catch (...) {
    }
  }
};

inline const char* kPredictPath = "/tensorflow.serving.PredictionService/Predict";

template <class H>
void def_grpc_front(py::module& m) {
  py::class_<GrpcFront>(m, "GrpcFront", py::module_local(),
                        "Native h2c gRPC PredictionService front door over a LiveServer (csrc/net/h2_server.h)")
      .def(py::init([](py::object live, int port, std::string host, int threads, py::object fallback,
                       int fallback_threads, int64_t max_message) {
             H& h = live.cast<H&>();
             auto f = std::make_unique<GrpcFront>();
             f->live = live;
             if (!fallback.is_none()) f->fb = std::make_shared<FallbackPool>(fallback.cast<py::function>(), fallback_threads);
             LiveServer* srv = h.srv.get();
             std::shared_ptr<FallbackPool> fb = f->fb;
             f->sp = std::make_shared<SubmitPool>(2);
             std::shared_ptr<SubmitPool> sp = f->sp;
             dtfs::net::H2Config cfg;
             cfg.host = host;
             cfg.port = port;
             cfg.threads = threads;
             cfg.max_message = max_message;
             auto handler = [srv, fb, sp](dtfs::net::GrpcCall&& call, dtfs::net::Responder r) {
               if (call.path != kPredictPath) {
                 if (fb) fb->push(std::move(call), std::move(r));
                 else r.reply(12, "method " + call.path + " is not implemented", "");
                 return;
               }
               auto msg = std::make_shared<std::string>(std::move(call.message));
               const int64_t dl = call.deadline_us;
               dtfs::runtime::Completion done = [r, fb, msg, dl](Reply&& rep) {
                             if (rep.code == dtfs::runtime::kOk) {
                               r.reply(0, std::string(), std::move(rep.response));
                             } else if ((rep.code == dtfs::runtime::kCallerPath || rep.code == dtfs::runtime::kOversize) &&
                                        fb) {
                               dtfs::net::GrpcCall c;
                               c.path = kPredictPath;
                               c.message = std::move(*msg);
                               c.deadline_us = dl;
                               fb->push(std::move(c), r);
                             } else {
                               r.reply(rep.code >= 1000 ? 13 : rep.code, std::move(rep.message), std::string());
                             }
                           };
               // never block the event loop (its other connections would stall
               // behind this call): the fast path admits in place, a full
               // batching queue goes to the submit pool
               if (srv->try_submit(reinterpret_cast<const uint8_t*>(msg->data()), msg->size(), dl, done)) return;
               auto task = [srv, msg, dl, done]() mutable {
                 srv->submit(reinterpret_cast<const uint8_t*>(msg->data()), msg->size(), dl, std::move(done));
               };
               if (!sp->push(std::move(task))) r.reply(8, "batching queue is full", "");
             };
             {
               py::gil_scoped_release nogil;
               f->h2 = std::make_unique<dtfs::net::H2GrpcServer>(cfg, handler);
             }
             return f.release();
           }),
           py::arg("live"), py::arg("port"), py::arg("host") = "0.0.0.0", py::arg("threads") = 4,
           py::arg("fallback") = py::none(), py::arg("fallback_threads") = 4, py::arg("max_message") = int64_t(64) << 20)
      .def_property_readonly("port", [](const GrpcFront& f) { return f.h2 ? f.h2->port() : 0; })
      .def("stop", &GrpcFront::stop)
      .def("stats", [](const GrpcFront& f) {
        const auto s = f.h2 ? f.h2->stats() : dtfs::net::H2Stats();
        py::dict o;
        o["connections"] = s.connections;
        o["open_connections"] = s.open_connections;
        o["calls"] = s.calls;
        o["replies"] = s.replies;
        o["dropped_replies"] = s.dropped_replies;
        o["resets"] = s.resets;
        o["protocol_errors"] = s.protocol_errors;
        o["paused_reads"] = s.paused_reads;
        o["bytes_in"] = s.bytes_in;
        o["bytes_out"] = s.bytes_out;
        o["blocking_submits_handed_off"] = f.sp ? f.sp->handed() : 0;
        return o;
      });
}

}  // namespace dtfs_live

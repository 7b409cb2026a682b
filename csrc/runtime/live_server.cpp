#include "live_server.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <exception>
#include <stdexcept>

#include "../wire/tensor_codec.h"
#include "batcher.h"  // now_us()
#include "narrow.h"
#include "trace.h"

namespace dtfs {
namespace runtime {

namespace {
int64_t align8(int64_t x) { return (x + 7) & ~int64_t(7); }
int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

std::string shape_str(const std::vector<int64_t>& s) {
  std::string o = "[";
  for (size_t i = 0; i < s.size(); ++i) o += (i ? ", " : "") + std::to_string(s[i]);
  return o + "]";
}
}  // namespace

LiveServer::LiveServer(StepBackend* backend, LiveConfig cfg, std::vector<std::pair<uint8_t*, int64_t>> arenas,
                       StepControl* ctl)
    : backend_(backend), cfg_(std::move(cfg)), ctl_(ctl), agree_(cfg_.liveness_only ? nullptr : ctl) {
  if (!backend_) throw std::invalid_argument("null StepBackend");
  const auto& bk = backend_->buckets();
  if (bk.empty() || !std::is_sorted(bk.begin(), bk.end()) || bk.front() <= 0)
    throw std::invalid_argument("buckets must be ascending positive row counts");
  const int S = backend_->slots();
  if (S < 1) throw std::invalid_argument("backend has no slots");
  cfg_.depth = std::max(1, std::min(cfg_.depth, S));
  max_rows_ = cfg_.max_batch_rows > 0 ? std::min(cfg_.max_batch_rows, bk.back()) : bk.back();
  if (int(arenas.size()) < cfg_.depth + 2)
    throw std::invalid_argument("need at least depth + 2 host arenas (one filling, one sealed, depth in flight)");
  int64_t cap = INT64_MAX;
  for (const auto& a : arenas) {
    if (!a.first || a.second <= kArenaPayloadOff + 4096) throw std::invalid_argument("bad host arena");
    cap = std::min(cap, a.second);
  }
  // arena_build appends, after the requests: 64-byte aligned scratch for
  // host-decoded typed fields, the row table, the varint chunk table and the
  // device-only decoded-id region; need_of() plans for the worst case of each
  arena_budget_ = cap - kArenaPayloadOff - 1024;
  arenas_.resize(arenas.size());
  for (size_t i = 0; i < arenas.size(); ++i) {
    arenas_[i].base = arenas[i].first;
    arenas_[i].capacity = arenas[i].second;
    free_.push_back(int(i));
  }
  slot_busy_.assign(size_t(S), 0);
  if (bk.size() > 0xffff) throw std::invalid_argument("too many buckets");
  // narrow_ids' AVX2 path multiplies with the low 32 bits of the modulo
  if (cfg_.narrow_modulo < 0 || cfg_.narrow_modulo >= (int64_t(1) << 31))
    throw std::invalid_argument("narrow_modulo must be in [0, 2^31)");
  if (cfg_.narrow_wts_cols < 0 || cfg_.narrow_wts_cols > cfg_.fields)
    throw std::invalid_argument("narrow_wts_cols must be in [0, fields]");
  paused_ = cfg_.start_paused;
  launcher_ = std::thread([this] { launcher_loop(); });
  completer_ = std::thread([this] { completer_loop(); });
  if (ctl_) watcher_ = std::thread([this] { watcher_loop(); });
}

LiveServer::~LiveServer() {
  try {
    close();
  } catch (...) {
  }
}

int64_t LiveServer::need_of(int64_t len, int64_t rows) const {
  const int64_t ne = rows * cfg_.fields;
  // bytes + typed-field scratch (int64 ids 8 B + fp32 weights 4 B per element,
  // or the GPU varint id region) + row table + varint chunk entries + alignment
  return align8(len) + 12 * ne + 8 * rows + 32 * (len / kVarintChunk + 2) + 256;
}

int LiveServer::bucket_for(int64_t rows) const {
  const auto& bk = backend_->buckets();
  for (size_t i = 0; i < bk.size(); ++i)
    if (bk[i] >= rows) return int(i);
  return int(bk.size()) - 1;
}

void LiveServer::submit(const uint8_t* data, size_t n, int64_t deadline_us, Completion done) {
  (void)admit(data, n, deadline_us, done, true);
}

bool LiveServer::try_submit(const uint8_t* data, size_t n, int64_t deadline_us, Completion& done) {
  return admit(data, n, deadline_us, done, false);
}

bool LiveServer::admit(const uint8_t* data, size_t n, int64_t deadline_us, Completion& done, bool wait) {
  auto reject = [&](int code, std::string msg) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      ++st_.rejected;
    }
    done(Reply{code, std::move(msg), std::string()});
    return true;
  };
  // framing + signature checks on the caller's thread (parallel across callers)
  wire::PredictRequestView v;
  std::string err;
  if (!wire::parse_predict_request(data, n, &v, &err, false))
    return reject(kInvalidArgument, "malformed PredictRequest: " + err);
  if (v.model_name != cfg_.model_name)
    return reject(kNotFound, "Servable not found for request: Latest(" + v.model_name + ")");
  if (v.has_version && (cfg_.version < 0 || v.version != cfg_.version))
    return reject(kNotFound, "Servable not found for request: Specific(" + v.model_name + ", " +
                                 std::to_string(v.version) + ")");
  if (!v.signature_name.empty() && v.signature_name != cfg_.signature_name)
    return reject(kInvalidArgument, "Serving signature name: \"" + v.signature_name +
                                        "\" not found in signature def of model " + cfg_.model_name);
  for (const auto& k : v.output_filter) {
    if (k == cfg_.output_key) continue;
    if (std::find(cfg_.caller_outputs.begin(), cfg_.caller_outputs.end(), k) != cfg_.caller_outputs.end())
      return reject(kCallerPath, "output " + k + " is produced by the general path");
    return reject(kInvalidArgument, "output tensor alias not found in signature: " + k);
  }
  const wire::TensorView* ti = v.find(cfg_.ids_key);
  const wire::TensorView* tw = v.find(cfg_.wts_key);
  if (!ti || !tw)
    return reject(kInvalidArgument, "input tensor alias not found in signature: " + (ti ? cfg_.wts_key : cfg_.ids_key));
  if (ti->unknown_rank || ti->shape.size() != 2 || ti->shape[1] != cfg_.fields || ti->shape[0] < 0)
    return reject(kInvalidArgument, cfg_.ids_key + " must have shape [B, " + std::to_string(cfg_.fields) + "], got " +
                                        shape_str(ti->shape));
  if (tw->shape != ti->shape)
    return reject(kInvalidArgument, cfg_.wts_key + " shape " + shape_str(tw->shape) + " != " + shape_str(ti->shape));
  if (ti->dtype != wire::DT_INT64 && ti->dtype != wire::DT_INT32)
    return reject(kInvalidArgument, cfg_.ids_key + " must be DT_INT64 or DT_INT32");
  const int64_t rows = ti->shape[0];
  wire::ModelSpecOut spec{cfg_.model_name, v.signature_name.empty() ? cfg_.signature_name : v.signature_name,
                          cfg_.version >= 0, cfg_.version};
  if (rows == 0) {
    wire::TensorOut t;
    t.key = cfg_.output_key;
    t.shape = {0};
    done(Reply{kOk, "", wire::encode_predict_response(spec, {t})});
    return true;
  }
  if (rows > max_rows_)
    return reject(kOversize, "request has " + std::to_string(rows) + " rows; a batch holds at most " +
                                 std::to_string(max_rows_));
  // narrowable: raw int64 ids + fp32 weights (tensor_content, or packed
  // float_val, which holds the same bytes)
  const int64_t ne = rows * cfg_.fields;
  const uint8_t* ids_src = nullptr;
  const uint8_t* wts_src = nullptr;
  if (cfg_.narrow_modulo > 0 && ti->dtype == wire::DT_INT64 && ti->content.n == size_t(ne) * 8 &&
      tw->dtype == wire::DT_FLOAT) {
    ids_src = ti->content.p;
    if (tw->content.n == size_t(ne) * 4) wts_src = tw->content.p;
    else if (tw->content.n == 0 && tw->value_fixed32 && tw->packed.size() == 1 && tw->unpacked.empty() &&
             tw->packed[0].n == size_t(ne) * 4)
      wts_src = tw->packed[0].p;
  }
  const bool narrow = ids_src && wts_src;
  const int64_t wcols = cfg_.narrow_wts_cols > 0 ? cfg_.narrow_wts_cols : cfg_.fields;  // narrow weights kept per row
  // the cheapest exact form of this request's weights (all 1.0: none travel)
  const int wkind = narrow ? classify_weights(wts_src, rows, cfg_.fields, wcols) : kWtsF32;
  const int64_t idb = narrow_id_bytes();  // 3-byte rows for tables of <= 2^24 rows
  const int64_t ids_bytes = idb == 3 ? 3 * ne + kNarrow24Slack : 4 * ne;
  const int64_t need = narrow ? align64(ids_bytes) + align64(4 * rows * wcols) + 8 * rows + 256 : need_of(int64_t(n), rows);
  if (need > arena_budget_) return reject(kOversize, "request does not fit one arena");

  const int64_t t0 = now_us();
  int a = -1;
  int64_t off = 0, pend_ids = 0, pend_wts = 0;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (broken_) {
      lk.unlock();
      return reject(kUnavailable, "server unavailable: " + error_);
    }
    if (closing_) {
      lk.unlock();
      return reject(kUnavailable, "server is shutting down");
    }
    if (pending_ >= cfg_.max_pending) {
      lk.unlock();
      return reject(kResourceExhausted, "batching queue is full");
    }
    bool blocked = false;
    for (;;) {
      if (open_ >= 0) {
        Arena& o = arenas_[size_t(open_)];
        if (o.rows + rows <= max_rows_ && o.need + need <= arena_budget_ &&
            int64_t(o.pend.size()) < kArenaMaxRequests)
          break;
        // the open batch is full for this request: seal it, take a fresh arena
        sealed_.push_back(open_);
        open_ = -1;
        cv_launch_.notify_all();
        continue;
      }
      if (!free_.empty()) {
        open_ = free_.front();
        free_.pop_front();
        continue;
      }
      // every arena is queued or in flight: wait for one (bounded by the deadline),
      // or tell a caller that must not block (an event-loop thread)
      if (!wait) return false;
      if (!blocked) {
        blocked = true;
        ++st_.blocked_submits;
      }
      auto ready = [&] { return broken_ || closing_ || open_ >= 0 || !free_.empty(); };
      if (deadline_us > 0) {
        const int64_t left = deadline_us - now_us();
        if (left <= 0 || !cv_space_.wait_for(lk, std::chrono::microseconds(left), ready)) {
          lk.unlock();
          return reject(kDeadlineExceeded, "request deadline exceeded while waiting for a batch slot");
        }
      } else {
        cv_space_.wait(lk, ready);
      }
      if (broken_ || closing_) {
        lk.unlock();
        return reject(kUnavailable, broken_ ? "server unavailable: " + error_ : "server is shutting down");
      }
    }
    a = open_;
    Arena& o = arenas_[size_t(a)];
    Pending p{0, int64_t(n), rows, deadline_us, t0, std::move(done)};
    if (narrow) {
      p.narrow = true;
      p.ids_off = align64(o.used);
      p.wts_off = align64(p.ids_off + ids_bytes);
      p.wkind = wkind;
      o.used = p.wts_off + wts_bytes_per(wkind) * rows * wcols;
      ++st_.narrowed;
      if (wkind == kWtsBf16) ++st_.narrowed_wts_bf16;
      if (wkind == kWtsOnes) ++st_.narrowed_wts_implicit;
    } else {
      off = p.off = o.used;
      o.used += align8(int64_t(n));
    }
    o.rows += rows;
    o.need += need;
    if (o.pend.empty()) {
      o.t_first = t0;
      cv_launch_.notify_all();  // eager dispatch / batch timeout start now
    }
    pend_ids = p.ids_off;
    pend_wts = p.wts_off;
    o.pend.push_back(std::move(p));
    ++o.writers;
    ++pending_;
    ++st_.submitted;
    if (o.rows >= max_rows_) {  // exactly full: hand it over without waiting for the next request
      sealed_.push_back(open_);
      open_ = -1;
      cv_launch_.notify_all();
    }
  }
  // the one copy of the request: into pinned memory the DMA engine reads
  uint8_t* payload = arenas_[size_t(a)].base + kArenaPayloadOff;
  if (narrow) {  // ... narrowed on the way (K0 on the host)
    if (idb == 3) narrow_ids24(ids_src, payload + pend_ids, ne, cfg_.narrow_modulo);
    else narrow_ids(ids_src, reinterpret_cast<int32_t*>(payload + pend_ids), ne, cfg_.narrow_modulo);
    // only the weight columns the model reads, in the cheapest exact form
    store_weights(wts_src, rows, cfg_.fields, wcols, wkind, payload + pend_wts);
  } else {
    std::memcpy(payload + off, data, n);
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    st_.copy_us += double(now_us() - t0);
    if (--arenas_[size_t(a)].writers == 0) cv_launch_.notify_all();
  }
  return true;
}

Reply LiveServer::predict(const uint8_t* data, size_t n, int64_t deadline_us) {
  std::mutex m;
  std::condition_variable cv;
  bool ready = false;
  Reply out;
  submit(data, n, deadline_us, [&](Reply&& r) {
    std::lock_guard<std::mutex> lk(m);
    out = std::move(r);
    ready = true;
    cv.notify_one();
  });
  std::unique_lock<std::mutex> lk(m);
  cv.wait(lk, [&] { return ready; });
  return out;
}

void LiveServer::fail_all(std::vector<Pending>& ps, int code, const std::string& msg) {
  for (auto& p : ps) {
    if (p.done) p.done(Reply{code, msg, std::string()});
    p.done = nullptr;
  }
  std::lock_guard<std::mutex> lk(mu_);
  pending_ -= int64_t(ps.size());
  st_.failed += int64_t(ps.size());
  if (code == kDeadlineExceeded) st_.expired += int64_t(ps.size());
}

void LiveServer::go_broken(const std::string& why) {
  std::vector<Pending> orphans;
  bool first = false;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!broken_) {
      first = true;
      broken_ = true;
      error_ = why;
    }
    // queued batches will never launch: answer them now (writers still
    // copying finish their memcpy; their Pending entries are taken here)
    for (int a : sealed_)
      for (auto& p : arenas_[size_t(a)].pend) orphans.push_back(std::move(p));
    for (int a : sealed_) arenas_[size_t(a)].pend.clear();
    if (open_ >= 0) {
      for (auto& p : arenas_[size_t(open_)].pend) orphans.push_back(std::move(p));
      arenas_[size_t(open_)].pend.clear();
    }
    cv_launch_.notify_all();
    cv_space_.notify_all();
    cv_done_.notify_all();
  }
  if (first) {
    try {
      backend_->abort();
    } catch (...) {
    }
  }
  fail_all(orphans, kUnavailable, "server unavailable: " + why);
}

void LiveServer::release(int a, int slot) {
  std::lock_guard<std::mutex> lk(mu_);
  Arena& ar = arenas_[size_t(a)];
  ar.used = ar.rows = ar.need = ar.t_first = 0;
  ar.pend.clear();
  free_.push_back(a);
  if (slot >= 0) {
    slot_busy_[size_t(slot)] = 0;
    --inflight_;
  }
  cv_space_.notify_all();
  cv_launch_.notify_all();
}

void LiveServer::launcher_loop() {
  const int S = backend_->slots();
  const int nb = int(backend_->buckets().size());
  for (;;) {
    int a = -1, slot = -1;
    uint64_t k = 0;            // cluster mode: the step index (identical on every rank)
    bool remote = false;       // cluster mode: another rank proposed the step
    int64_t arena_rows = 0;
    std::vector<Pending> pend;
    bool stop = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      // a free slot first: while the device is busy, requests keep filling the
      // open batch (fuller steps under load)
      auto slot_free = [&] { return inflight_ < cfg_.depth && !slot_busy_[size_t(next_slot_)]; };
      auto drained = [&] { return closing_ && sealed_.empty() && (open_ < 0 || arenas_[size_t(open_)].pend.empty()); };
      if (!agree_) {
        cv_launch_.wait(lk, [&] { return broken_ || (!paused_ && (drained() || slot_free())) || (paused_ && closing_); });
        if (paused_ && closing_) break;  // never started: nothing was launched
        if (broken_ || !slot_free()) break;
      }
      for (;;) {
        if (broken_) break;
        if (paused_) {
          if (closing_) {  // never started: nothing was launched
            stop = true;
            break;
          }
          cv_launch_.wait(lk);
          continue;
        }
        const int64_t now = now_us();
        int64_t wake = 0;
        // does this rank have a batch to run now?
        bool local = !sealed_.empty();
        if (!local && open_ >= 0 && !arenas_[size_t(open_)].pend.empty()) {
          const Arena& o = arenas_[size_t(open_)];
          const bool idle = cfg_.eager_when_idle && inflight_ == 0;
          if (closing_ || idle || now >= o.t_first + cfg_.batch_timeout_us) local = true;
          else wake = o.t_first + cfg_.batch_timeout_us;
        }
        if (!agree_) {
          if (!sealed_.empty()) {
            a = sealed_.front();
            sealed_.pop_front();
            ++st_.full_steps;
            break;
          }
          if (local) {
            const bool idle = cfg_.eager_when_idle && inflight_ == 0;
            a = open_;
            open_ = -1;
            ++(idle ? st_.eager_steps : st_.timeout_steps);
            break;
          }
          if (closing_) {  // drained
            stop = true;
            break;
          }
        } else {
          // cluster mode: launch step k when this rank has a batch for it or
          // another rank proposed it; leave once every rank is closing and no
          // step is pending (read closing flags BEFORE `proposed`: a rank
          // proposes its last step before it raises its closing flag)
          k = uint64_t(steps_launched_);
          if (drained() && !closing_posted_) {
            closing_posted_ = true;
            agree_->set_closing(true);
          }
          if (closing_posted_ && agree_->all_closing() && agree_->proposed() <= k) {
            stop = true;
            break;
          }
          remote = agree_->proposed() > k;
          if ((remote || local) && slot_free()) {
            if (!sealed_.empty()) {
              a = sealed_.front();
              sealed_.pop_front();
              ++st_.full_steps;
            } else if (open_ >= 0 && !arenas_[size_t(open_)].pend.empty()) {
              a = open_;
              open_ = -1;
              ++(local ? st_.timeout_steps : st_.joined_steps);
            } else if (!free_.empty() || open_ >= 0) {
              // nothing queued here: an empty contribution to another rank's step
              if (open_ >= 0) {
                a = open_;
                open_ = -1;
              } else {
                a = free_.front();
                free_.pop_front();
              }
              ++st_.empty_steps;
            }
            if (a >= 0) {
              if (!remote) ++st_.proposed_steps;
              break;
            }
          }
        }
        // nothing to launch yet: sleep until a submit / slot release / the
        // batch timeout, or (cluster) a proposal, which the watcher relays
        if (agree_ && !(remote || local)) {
          launcher_idle_.store(true, std::memory_order_seq_cst);
          agree_->set_idle(true);
          // re-check after announcing idleness (seq_cst against propose())
          if (agree_->proposed() <= k && !broken_) {
            if (wake > 0) cv_launch_.wait_for(lk, std::chrono::microseconds(std::max<int64_t>(1, wake - now)));
            else cv_launch_.wait_for(lk, std::chrono::microseconds(cfg_.heartbeat_us));
          }
          agree_->set_idle(false);
          launcher_idle_.store(false, std::memory_order_seq_cst);
        } else if (agree_) {
          // a step to launch but no free slot / arena yet: release() notifies
          cv_launch_.wait_for(lk, std::chrono::microseconds(cfg_.heartbeat_us));
        } else if (wake > 0) {
          cv_launch_.wait_for(lk, std::chrono::microseconds(std::max<int64_t>(1, wake - now)));
        } else {
          cv_launch_.wait(lk);
        }
      }
      if (broken_ || stop) break;
      // writers that reserved space in this batch finish their copies first
      cv_launch_.wait(lk, [&] { return arenas_[size_t(a)].writers == 0; });
      pend = std::move(arenas_[size_t(a)].pend);
      arenas_[size_t(a)].pend.clear();
      arena_rows = arenas_[size_t(a)].rows;
      slot = next_slot_;
      slot_busy_[size_t(slot)] = 1;
      next_slot_ = (next_slot_ + 1) % S;
      ++inflight_;
      ++steps_launched_;
    }
    int agreed = -1;
    if (agree_) {
      // agree on step k's bucket with every rank (step_control.h)
      const int mine = arena_rows > 0 ? bucket_for(arena_rows) : 0;
      std::string gerr;
      int b = -1;
      try {
        trace::Range tr("live_agree");
        if (!remote) agree_->propose(k);
        agree_->post(k, mine);
        b = agree_->gather(k, cfg_.step_timeout_us, &gerr);
      } catch (const std::exception& e) {
        gerr = e.what();
      }
      if (b < 0 || b >= nb) {
        const std::string why = "step agreement failed: " + (b >= nb ? std::string("bucket out of range") : gerr);
        fail_all(pend, kUnavailable, "server unavailable: " + why);
        release(a, slot);
        agree_->mark_broken(agree_->rank());
        go_broken(why);
        break;
      }
      agreed = b;
    }
    // requests whose deadline passed while queued are answered, not computed
    const int64_t t0 = now_us();
    std::vector<Pending> live, expired;
    live.reserve(pend.size());
    for (auto& p : pend) (p.deadline_us > 0 && t0 > p.deadline_us ? expired : live).push_back(std::move(p));
    if (!expired.empty()) fail_all(expired, kDeadlineExceeded, "request deadline exceeded while queued");
    std::vector<ArenaItem> items(live.size());
    for (size_t i = 0; i < live.size(); ++i) {
      const Pending& p = live[i];
      ArenaItem& it = items[i];
      it.off = p.off;
      it.len = p.len;
      it.narrow = p.narrow;
      it.rows = p.rows;
      it.ids_off = p.ids_off;
      it.wts_off = p.wts_off;
      it.wkind = p.wkind;
    }
    Arena& ar = arenas_[size_t(a)];
    ArenaBatch batch;
    try {
      trace::Range tr("live_build");
      batch = arena_build_items(ar.base, ar.capacity, items, cfg_.ids_key, cfg_.wts_key, cfg_.fields, max_rows_,
                                cfg_.varint_chunks, cfg_.narrow_wts_cols, narrow_id_bytes());
    } catch (const std::exception& e) {
      fail_all(live, kInternal, std::string("batch build failed: ") + e.what());
      if (agree_) {  // the other ranks launch step k: this rank cannot skip it
        const std::string why = std::string("batch build failed in a cluster step: ") + e.what();
        release(a, slot);
        agree_->mark_broken(agree_->rank());
        go_broken(why);
        break;
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        --steps_launched_;
      }
      release(a, slot);
      continue;
    }
    const int64_t t1 = now_us();
    if (batch.n_valid == 0 && !agree_) {
      // nothing to compute: every request was malformed (or none left)
      for (size_t i = 0; i < live.size(); ++i)
        if (live[i].done) live[i].done(Reply{kInvalidArgument, batch.errors[i], std::string()});
      {
        std::lock_guard<std::mutex> lk(mu_);
        pending_ -= int64_t(live.size());
        st_.failed += int64_t(live.size());
        --steps_launched_;
      }
      release(a, slot);
      continue;
    }
    const int b = agree_ ? agreed : bucket_for(batch.total_rows);
    try {
      trace::Range tr("live_launch");
      backend_->launch(slot, b, ar.base, batch);
    } catch (const std::exception& e) {
      const std::string why = std::string("step launch failed: ") + e.what();
      fail_all(live, kUnavailable, why);
      release(a, slot);
      if (agree_) agree_->mark_broken(agree_->rank());
      go_broken(why);
      break;
    }
    const int64_t t2 = now_us();
    std::lock_guard<std::mutex> lk(mu_);
    st_.build_us += double(t1 - t0);
    st_.launch_us += double(t2 - t1);
    ++st_.steps;
    st_.rows += batch.total_rows;
    st_.padded_rows += backend_->buckets()[size_t(std::min(b, nb - 1))];
    q_done_.push_back(InFlight{a, slot, b, std::move(batch), std::move(live), t2});
    cv_done_.notify_all();
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    launcher_exited_ = true;
    closing_ = true;  // a stopped launcher admits nothing more
    cv_done_.notify_all();
    cv_space_.notify_all();
  }
  if (agree_ && !closing_posted_) agree_->set_closing(true);
  // whatever is still queued will not be launched
  std::vector<Pending> orphans;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (int x : sealed_) {
      for (auto& p : arenas_[size_t(x)].pend) orphans.push_back(std::move(p));
      arenas_[size_t(x)].pend.clear();
    }
    if (open_ >= 0) {
      for (auto& p : arenas_[size_t(open_)].pend) orphans.push_back(std::move(p));
      arenas_[size_t(open_)].pend.clear();
    }
  }
  if (!orphans.empty())
    fail_all(orphans, kUnavailable, broken_ ? "server unavailable: " + error_ : "server stopped before the request ran");
}

void LiveServer::watcher_loop() {
  for (;;) {
    const uint32_t seen = ctl_->bell();
    ctl_->heartbeat();
    if (!broken_) {
      // any broken flag breaks this server, this rank's own included: the
      // front door marks the cluster broken from Python on a communicator
      // error (serving/cluster.py _watch) while this server may be idle, and
      // only a broken server starts the rebuild
      const int by = ctl_->broken_by();
      if (by >= 0) {
        go_broken(by == ctl_->rank() ? std::string("this rank gave up on the cluster")
                                     : "rank " + std::to_string(by) + " gave up on the cluster");
      } else {
        const int silent = ctl_->silent_peer(cfg_.peer_timeout_us);
        if (silent >= 0) {
          ctl_->mark_broken(ctl_->rank());
          go_broken(ctl_->process_gone(silent)
                        ? "rank " + std::to_string(silent) + " exited"
                        : "rank " + std::to_string(silent) + " stopped answering (no heartbeat for " +
                              std::to_string(cfg_.peer_timeout_us / 1000) + " ms)");
        }
      }
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (watcher_stop_) break;
      if (launcher_idle_.load(std::memory_order_seq_cst) || broken_) cv_launch_.notify_all();
    }
    ctl_->wait_bell(seen, cfg_.heartbeat_us);
  }
}

void LiveServer::completer_loop() {
  wire::ModelSpecOut spec{cfg_.model_name, cfg_.signature_name, cfg_.version >= 0, cfg_.version};
  for (;;) {
    InFlight f;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_done_.wait(lk, [&] { return !q_done_.empty() || launcher_exited_; });
      if (q_done_.empty()) break;
      f = std::move(q_done_.front());
      q_done_.pop_front();
    }
    const int64_t t0 = now_us();
    std::string err;
    bool ok = false;
    try {
      trace::Range tr("live_wait");
      // after a failure the remaining steps get a short grace period only
      ok = backend_->wait(f.slot, broken_ ? 200'000 : cfg_.step_timeout_us, &err);
      if (!ok && err.empty()) err = "step did not finish within the step timeout";
    } catch (const std::exception& e) {
      err = e.what();
    }
    const int64_t t1 = now_us();
    if (!ok) {
      const std::string why = "GPU step failed: " + err;
      fail_all(f.pend, kUnavailable, "server unavailable: " + why);
      go_broken(why);
      release(f.arena, f.slot);
      continue;
    }
    const float* sc = backend_->scores(f.slot, f.bucket);
    const int64_t sc_len = backend_->scores_len(f.slot, f.bucket);
    int64_t n_ok = 0, n_bad = 0;
    {
      trace::Range tr("live_encode");
      for (size_t i = 0; i < f.pend.size(); ++i) {
        Pending& p = f.pend[i];
        Reply r;
        const std::string& e = f.batch.errors[i];
        if (!e.empty()) {
          r.code = kInvalidArgument;
          r.message = e;
          ++n_bad;
        } else if (f.batch.offsets[i] + f.batch.rows[i] > sc_len) {
          r.code = kInternal;
          r.message = "scores buffer smaller than the batch";
          ++n_bad;
        } else {
          wire::TensorOut t;
          t.key = cfg_.output_key;
          t.dtype = wire::DT_FLOAT;
          t.shape = {f.batch.rows[i]};
          t.data = sc + f.batch.offsets[i];
          t.n = f.batch.rows[i];
          r.response = wire::encode_predict_response(spec, {t});
          ++n_ok;
        }
        r.t_arrive = p.t_arrive;
        r.t_launch = f.t_launch;
        r.t_done = t1;
        r.t_encoded = now_us();
        if (p.done) p.done(std::move(r));
        p.done = nullptr;
      }
    }
    const int64_t t2 = now_us();
    {
      std::lock_guard<std::mutex> lk(mu_);
      pending_ -= int64_t(f.pend.size());
      st_.completed += n_ok;
      st_.failed += n_bad;
      st_.wait_us += double(t1 - t0);
      st_.encode_us += double(t2 - t1);
    }
    release(f.arena, f.slot);
  }
}

void LiveServer::resume() {
  std::lock_guard<std::mutex> lk(mu_);
  paused_ = false;
  cv_launch_.notify_all();
}

void LiveServer::close() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    closing_ = true;
    cv_launch_.notify_all();
    cv_space_.notify_all();
  }
  // cluster mode: the launcher keeps joining the other ranks' steps until
  // every rank is closing (the watcher keeps the heartbeat going meanwhile)
  if (launcher_.joinable()) launcher_.join();
  if (completer_.joinable()) completer_.join();
  if (watcher_.joinable()) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      watcher_stop_ = true;
    }
    ctl_->ring();
    watcher_.join();
  }
}

LiveStats LiveServer::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  LiveStats s = st_;
  s.broken = broken_;
  s.error = error_;
  return s;
}

}  // namespace runtime
}  // namespace dtfs

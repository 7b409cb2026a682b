#include "arena.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <stdexcept>

#include "../wire/tensor_codec.h"
#include "thread_pool.h"

namespace dtfs {
namespace runtime {

std::vector<Span> arena_place(uint8_t* arena, int64_t capacity, const std::vector<std::pair<const char*, size_t>>& reqs,
                              int64_t start) {
  std::vector<Span> spans(reqs.size());
  int64_t off = start;
  for (size_t i = 0; i < reqs.size(); ++i) {
    spans[i] = {off, int64_t(reqs[i].second)};
    off += (int64_t(reqs[i].second) + 7) & ~int64_t(7);
  }
  if (kArenaPayloadOff + off > capacity) throw std::invalid_argument("arena too small for the batch");
  uint8_t* payload = arena + kArenaPayloadOff;
  ThreadPool::global().parallel_for(int64_t(reqs.size()), [&](int64_t i) {
    std::memcpy(payload + spans[i].first, reqs[i].first, reqs[i].second);
  });
  return spans;
}

ArenaBatch arena_build(uint8_t* base, int64_t capacity, const std::vector<Span>& spans, const std::string& ids_key,
                       const std::string& wts_key, int64_t fields, int64_t max_rows) {
  if (int64_t(spans.size()) > kArenaMaxRequests) throw std::invalid_argument("too many requests for one arena");
  uint8_t* payload = base + kArenaPayloadOff;
  const int64_t cap = capacity - kArenaPayloadOff;
  ArenaBatch out;
  const size_t n = spans.size();
  out.rows.assign(n, 0);
  out.offsets.assign(n, 0);
  out.errors.assign(n, std::string());
  int64_t end = 0;
  for (const auto& s : spans) {
    if (s.first < 0 || s.second < 0 || s.first + s.second > cap) throw std::invalid_argument("request span outside arena");
    end = std::max(end, s.first + s.second);
  }
  int64_t scratch = (end + 63) & ~int64_t(63);
  int64_t* desc = reinterpret_cast<int64_t*>(base + 64);
  struct Job {
    int64_t req;
    const wire::TensorView *ti, *tw;
    int64_t ne, ids_off, wts_off, ids_scratch, wts_scratch;
  };
  std::vector<Job> jobs;
  std::vector<wire::PredictRequestView> views(n);
  int64_t nd = 0, row = 0;
  for (size_t i = 0; i < n; ++i) {
    std::string err;
    auto& v = views[i];
    if (!wire::parse_predict_request(payload + spans[i].first, size_t(spans[i].second), &v, &err)) {
      out.errors[i] = "malformed PredictRequest: " + err;
      continue;
    }
    const wire::TensorView* ti = v.find(ids_key);
    const wire::TensorView* tw = v.find(wts_key);
    if (!ti || !tw) {
      out.errors[i] = "input '" + (ti ? wts_key : ids_key) + "' missing";
      continue;
    }
    if (ti->unknown_rank || ti->shape.size() != 2 || ti->shape[1] != fields || ti->shape[0] < 0 ||
        tw->shape != ti->shape) {
      out.errors[i] = "inputs must have shape [B, " + std::to_string(fields) + "]";
      continue;
    }
    const int64_t rows = ti->shape[0], ne = rows * fields;
    if (row + rows > max_rows) {
      out.errors[i] = "batch exceeds the arena's row capacity";
      continue;
    }
    const bool ids_raw = ti->content.n > 0 && ti->dtype == wire::DT_INT64 && ti->content.n == size_t(ne) * 8;
    const bool wts_raw = tw->content.n > 0 && tw->dtype == wire::DT_FLOAT && tw->content.n == size_t(ne) * 4;
    if ((!ids_raw && ti->num_values > ne) || (!wts_raw && tw->num_values > ne)) {
      out.errors[i] = "more values than the tensor shape holds";
      continue;
    }
    // plan: raw payloads are referenced in place; the rest get scratch space
    // and are decoded below, in parallel
    const int64_t need =
        (ids_raw ? 0 : ((ne * 8 + 63) & ~int64_t(63))) + (wts_raw ? 0 : ((ne * 4 + 63) & ~int64_t(63)));
    if (scratch + need > cap) {
      out.errors[i] = "arena scratch exhausted";
      continue;
    }
    Job j{int64_t(i), ti, tw, ne, ids_raw ? int64_t(ti->content.p - payload) : -1,
          wts_raw ? int64_t(tw->content.p - payload) : -1, 0, 0};
    if (!ids_raw) {
      j.ids_scratch = scratch;
      scratch += (ne * 8 + 63) & ~int64_t(63);
    }
    if (!wts_raw) {
      j.wts_scratch = scratch;
      scratch += (ne * 4 + 63) & ~int64_t(63);
    }
    jobs.push_back(j);
    desc[4 * nd + 0] = ids_raw ? j.ids_off : j.ids_scratch;
    desc[4 * nd + 1] = wts_raw ? j.wts_off : j.wts_scratch;
    desc[4 * nd + 2] = rows;
    desc[4 * nd + 3] = row;
    ++nd;
    out.rows[i] = rows;
    out.offsets[i] = row;
    row += rows;
  }
  // typed-field (varint / float_val) decode, one request per pool task
  std::vector<std::string> errs(jobs.size());
  bool any_typed = false;
  for (const Job& j : jobs) any_typed |= (j.ids_off < 0 || j.wts_off < 0);
  if (any_typed) {
    ThreadPool::global().parallel_for(int64_t(jobs.size()), [&](int64_t k) {
      const Job& j = jobs[k];
      std::string err;
      if (j.ids_off < 0) {
        wire::DecodeOpts o;
        o.dst = wire::DstType::I64;
        if (!wire::decode_into(*j.ti, payload + j.ids_scratch, j.ne, o, &err)) errs[k] = "input '" + ids_key + "': " + err;
      }
      if (j.wts_off < 0 && errs[k].empty()) {
        wire::DecodeOpts o;
        o.dst = wire::DstType::F32;
        if (!wire::decode_into(*j.tw, payload + j.wts_scratch, j.ne, o, &err)) errs[k] = "input '" + wts_key + "': " + err;
      }
    });
  }
  for (size_t k = 0; k < jobs.size(); ++k) {
    if (jobs[k].ids_off < 0) ++out.n_decoded;
    // decode failed late: its rows stay in the batch (scored, dropped), the
    // request itself is answered with the error
    if (!errs[k].empty()) out.errors[jobs[k].req] = errs[k];
  }
  // per-row offset table: {ids_off, wts_off} int32 (payload-relative)
  const int64_t rt = (std::max(end, scratch) + 63) & ~int64_t(63);
  if (rt + row * 8 > cap) throw std::invalid_argument("arena too small for the row table");
  if (rt + row * 8 > int64_t(INT32_MAX)) throw std::invalid_argument("arena payload exceeds 2 GiB");
  int32_t* tab = reinterpret_cast<int32_t*>(payload + rt);
  for (int64_t d = 0; d < nd; ++d) {
    const int64_t io = desc[4 * d + 0], wo = desc[4 * d + 1], rows = desc[4 * d + 2], r0 = desc[4 * d + 3];
    for (int64_t r = 0; r < rows; ++r) {
      tab[2 * (r0 + r) + 0] = int32_t(io + r * 8 * fields);
      tab[2 * (r0 + r) + 1] = int32_t(wo + r * 4 * fields);
    }
  }
  *reinterpret_cast<int32_t*>(base) = int32_t(nd);
  *reinterpret_cast<int64_t*>(base + 8) = row;
  *reinterpret_cast<int64_t*>(base + 16) = rt;
  out.total_rows = row;
  out.n_valid = nd;
  out.used_bytes = kArenaPayloadOff + rt + row * 8;
  return out;
}

void arena_unpack_cpu(const uint8_t* base, uint8_t* dst, int64_t B, int64_t W, int64_t fields) {
  const int32_t n = std::min<int32_t>(*reinterpret_cast<const int32_t*>(base), int32_t(kArenaMaxRequests));
  const int64_t* desc = reinterpret_cast<const int64_t*>(base + 64);
  const uint8_t* payload = base + kArenaPayloadOff;
  std::memset(dst, 0, size_t(B * W * 8));
  for (int32_t i = 0; i < n; ++i) {
    for (int64_t r = 0; r < desc[4 * i + 2]; ++r) {
      const int64_t row = desc[4 * i + 3] + r;
      if (row >= B) break;
      std::memcpy(dst + row * W * 8, payload + desc[4 * i + 0] + r * 8 * fields, size_t(8 * fields));
      std::memcpy(dst + row * W * 8 + 8 * fields, payload + desc[4 * i + 1] + r * 4 * fields, size_t(4 * fields));
    }
  }
}

}  // namespace runtime
}  // namespace dtfs

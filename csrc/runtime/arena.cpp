#include "arena.h"
#include "narrow.h"

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


int64_t arena_varint_capacity(int64_t max_rows, int64_t fields, int64_t max_requests) {
  // <= 10 bytes per int64 varint, plus one partial chunk per request
  return (max_rows * fields * 10 + kVarintChunk - 1) / kVarintChunk + max_requests;
}

void arena_varint_cpu(uint8_t* base) {
  const int64_t vt = *reinterpret_cast<const int64_t*>(base + 24);
  const int32_t n = *reinterpret_cast<const int32_t*>(base + 32);
  uint8_t* payload = base + kArenaPayloadOff;
  const VarintChunk* tab = reinterpret_cast<const VarintChunk*>(payload + vt);
  for (int32_t c = 0; c < n; ++c) {
    const VarintChunk& ch = tab[c];
    const uint8_t* src = payload + ch.src_off;
    int64_t* dst = reinterpret_cast<int64_t*>(payload + ch.dst_off);
    int64_t idx = ch.first_idx;
    for (int32_t j = 0; j < ch.len; ++j) {
      if (src[j] & 0x80) continue;
      uint64_t v = src[j] & 0x7f;
      for (int64_t k = int64_t(j) - 1, steps = 0; k >= -int64_t(ch.blob_lo) && steps < 9; --k, ++steps) {
        if ((src[k] & 0x80) == 0) break;
        v = (v << 7) | (src[k] & 0x7f);
      }
      if (idx < ch.n_values) dst[idx] = int64_t(v);
      ++idx;
    }
  }
}

ArenaBatch arena_build(uint8_t* base, int64_t capacity, const std::vector<Span>& spans, const std::string& ids_key,
                       const std::string& wts_key, int64_t fields, int64_t max_rows, int64_t varint_chunks) {
  std::vector<ArenaItem> items(spans.size());
  for (size_t i = 0; i < spans.size(); ++i) {
    items[i].off = spans[i].first;
    items[i].len = spans[i].second;
  }
  return arena_build_items(base, capacity, items, ids_key, wts_key, fields, max_rows, varint_chunks);
}

ArenaBatch arena_build_items(uint8_t* base, int64_t capacity, const std::vector<ArenaItem>& items,
                             const std::string& ids_key, const std::string& wts_key, int64_t fields, int64_t max_rows,
                             int64_t varint_chunks, int64_t narrow_wcols, int64_t narrow_id_bytes) {
  if (int64_t(items.size()) > kArenaMaxRequests) throw std::invalid_argument("too many requests for one arena");
  if (narrow_wcols < 0 || narrow_wcols > fields) throw std::invalid_argument("narrow_wcols must be in [0, fields]");
  if (narrow_id_bytes != 3 && narrow_id_bytes != 4) throw std::invalid_argument("narrow_id_bytes must be 3 or 4");
  const int64_t idb = narrow_id_bytes;
  const int64_t wcols = narrow_wcols > 0 ? narrow_wcols : fields;  // weights per narrowed row
  uint8_t* payload = base + kArenaPayloadOff;
  const int64_t cap = capacity - kArenaPayloadOff;
  ArenaBatch out;
  const size_t n = items.size();
  out.rows.assign(n, 0);
  out.offsets.assign(n, 0);
  out.errors.assign(n, std::string());
  std::vector<Span> spans(n);
  int64_t end = 0;
  for (size_t i = 0; i < n; ++i) {
    const ArenaItem& it = items[i];
    if (it.narrow) {
      const int64_t ne = it.rows * fields;
      const int64_t nwb = it.rows * wcols * wts_bytes_per(it.wkind);
      if (it.rows < 0 || it.ids_off < 0 || it.wts_off < 0 || it.ids_off % 4 || it.wts_off % 4 ||
          it.wkind < kWtsF32 || it.wkind > kWtsOnes || it.ids_off + idb * ne + 4 > cap || it.wts_off + nwb > cap ||
          it.wts_off >= (int64_t(1) << kWtsKindShift))
        throw std::invalid_argument("narrow request outside arena");
      end = std::max(end, std::max(it.ids_off + idb * ne + 4, it.wts_off + nwb));  // +4: a reader's 4-byte load of the last 3-byte id
      continue;
    }
    spans[i] = {it.off, it.len};
    if (it.off < 0 || it.len < 0 || it.off + it.len > cap) throw std::invalid_argument("request span outside arena");
    end = std::max(end, it.off + it.len);
  }
  int64_t scratch = (end + 63) & ~int64_t(63);
  int64_t* desc = reinterpret_cast<int64_t*>(base + 64);
  struct Job {
    int64_t req;
    const wire::TensorView *ti, *tw;
    int64_t ne, ids_off, wts_off, ids_scratch, wts_scratch;
  };
  std::vector<Job> jobs;
  struct GpuJob {
    int64_t desc, src_off, len, ne, req;
  };
  std::vector<GpuJob> gjobs;
  int64_t n_chunks = 0;
  std::vector<wire::PredictRequestView> views(n);
  int64_t nd = 0, row = 0;
  // framing parse, one request per pool task (packed varint fields are
  // counted here: ~6 bytes per id for ids over 2^40)
  // Packed varint ids are counted once, per GPU decode chunk (the counts
  // validate the value count and give each chunk its first index).
  std::vector<char> parsed_ok(n, 0);
  std::vector<std::string> perr(n);
  std::vector<std::vector<int32_t>> chunk_counts(n);
  // framing only (~1 us per request), then the counting on the pool for the
  // requests that have uncounted varints
  std::vector<int64_t> to_count;
  for (size_t i = 0; i < n; ++i) {
    if (items[i].narrow) continue;
    parsed_ok[i] = wire::parse_predict_request(payload + spans[i].first, size_t(spans[i].second), &views[i], &perr[i],
                                               false);
    if (!parsed_ok[i]) continue;
    for (const auto& kv : views[i].inputs)
      if (kv.second.num_values < 0) {
        to_count.push_back(int64_t(i));
        break;
      }
  }
  auto count_one = [&](int64_t i) {
    for (auto& kv : views[size_t(i)].inputs) {
      wire::TensorView& t = kv.second;
      if (t.num_values >= 0) continue;
      int64_t total = int64_t(t.unpacked.size());
      if (kv.first == ids_key && t.packed.size() == 1) {
        auto& cc = chunk_counts[size_t(i)];
        const wire::Span& sp = t.packed[0];
        for (size_t lo = 0; lo < sp.n; lo += size_t(kVarintChunk)) {
          cc.push_back(int32_t(wire::count_varint_terminators(sp.p + lo, std::min(size_t(kVarintChunk), sp.n - lo))));
          total += cc.back();
        }
      } else {
        for (const wire::Span& sp : t.packed) total += wire::count_varint_terminators(sp.p, sp.n);
      }
      t.num_values = total;
    }
  };
  if (to_count.size() > 1)
    ThreadPool::global().parallel_for(int64_t(to_count.size()), [&](int64_t k) { count_one(to_count[size_t(k)]); });
  else if (!to_count.empty())
    count_one(to_count[0]);
  for (size_t i = 0; i < n; ++i) {
    if (items[i].narrow) {
      const int64_t rows = items[i].rows;
      if (row + rows > max_rows) {
        out.errors[i] = "batch exceeds the arena's row capacity";
        continue;
      }
      desc[4 * nd + 0] = items[i].ids_off | kNarrowFlag;
      desc[4 * nd + 1] = items[i].wts_off | (int64_t(items[i].wkind) << kWtsKindShift);
      desc[4 * nd + 2] = rows;
      desc[4 * nd + 3] = row;
      ++nd;
      out.rows[i] = rows;
      out.offsets[i] = row;
      row += rows;
      continue;
    }
    auto& v = views[i];
    if (!parsed_ok[i]) {
      out.errors[i] = "malformed PredictRequest: " + perr[i];
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
    // packed float_val holds the same little-endian bytes as tensor_content
    const bool wts_packed = tw->content.n == 0 && tw->dtype == wire::DT_FLOAT && tw->value_fixed32 &&
                            tw->packed.size() == 1 && tw->unpacked.empty() && tw->packed[0].n == size_t(ne) * 4;
    const bool wts_raw = wts_packed ||
                         (tw->content.n > 0 && tw->dtype == wire::DT_FLOAT && tw->content.n == size_t(ne) * 4);
    const uint8_t* wts_bytes = wts_packed ? tw->packed[0].p : tw->content.p;
    // packed varint ids -> GPU decode (one run of varints, exactly ne values)
    const int64_t ids_chunks = (!ids_raw && ti->content.n == 0 && ti->dtype == wire::DT_INT64 &&
                                ti->value_packed_varint && ti->packed.size() == 1 && ti->unpacked.empty() &&
                                ti->num_values == ne && ne > 0)
                                   ? (int64_t(ti->packed[0].n) + kVarintChunk - 1) / kVarintChunk
                                   : 0;
    const bool ids_gpu = ids_chunks > 0 && n_chunks + ids_chunks <= varint_chunks;
    if ((!ids_raw && ti->num_values > ne) || (!wts_raw && tw->num_values > ne)) {
      out.errors[i] = "more values than the tensor shape holds";
      continue;
    }
    // plan: raw payloads are referenced in place; the rest get scratch space
    // and are decoded below, in parallel
    const int64_t need = (ids_raw || ids_gpu ? 0 : ((ne * 8 + 63) & ~int64_t(63))) +
                         (wts_raw ? 0 : ((ne * 4 + 63) & ~int64_t(63)));
    if (scratch + need > cap) {
      out.errors[i] = "arena scratch exhausted";
      continue;
    }
    Job j{int64_t(i), ti, tw, ne, ids_raw ? int64_t(ti->content.p - payload) : (ids_gpu ? 0 : -1),
          wts_raw ? int64_t(wts_bytes - payload) : -1, 0, 0};
    if (ids_gpu) {
      gjobs.push_back({nd, int64_t(ti->packed[0].p - payload), int64_t(ti->packed[0].n), ne, int64_t(i)});
      n_chunks += ids_chunks;
    } else if (!ids_raw) {
      j.ids_scratch = scratch;
      scratch += (ne * 8 + 63) & ~int64_t(63);
    }
    if (!wts_raw) {
      j.wts_scratch = scratch;
      scratch += (ne * 4 + 63) & ~int64_t(63);
    }
    jobs.push_back(j);
    desc[4 * nd + 0] = ids_raw ? j.ids_off : (ids_gpu ? -1 : j.ids_scratch);
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
  // per-row offset table: {ids_off, wts_off} int32 (payload-relative), then
  // the varint chunk table (both copied to the GPU), then the device-only
  // region the varint kernel decodes ids into
  const int64_t rt = (std::max(end, scratch) + 63) & ~int64_t(63);
  const int64_t vt = (rt + row * 8 + 63) & ~int64_t(63);
  const int64_t vt_end = vt + n_chunks * int64_t(sizeof(VarintChunk));
  int64_t dec = (vt_end + 63) & ~int64_t(63);
  for (const GpuJob& g : gjobs) dec += g.ne * 8;
  if (std::max(vt_end, dec) > cap) throw std::invalid_argument("arena too small for the row table");
  if (std::max(vt_end, dec) > int64_t(INT32_MAX)) throw std::invalid_argument("arena payload exceeds 2 GiB");
  {
    // chunk tables, one request per pool task
    VarintChunk* vtab = reinterpret_cast<VarintChunk*>(payload + vt);
    std::vector<int64_t> first_chunk(gjobs.size()), dst(gjobs.size());
    int64_t d = (vt_end + 63) & ~int64_t(63), c = 0;
    for (size_t k = 0; k < gjobs.size(); ++k) {
      desc[4 * gjobs[k].desc + 0] = d;
      dst[k] = d;
      first_chunk[k] = c;
      c += (gjobs[k].len + kVarintChunk - 1) / kVarintChunk;
      d += gjobs[k].ne * 8;
    }
    for (size_t k = 0; k < gjobs.size(); ++k) {
      const GpuJob& g = gjobs[k];
      const auto& cc = chunk_counts[size_t(g.req)];
      int64_t before = 0, ci = first_chunk[k];
      for (int64_t lo = 0, q = 0; lo < g.len; lo += kVarintChunk, ++q) {
        VarintChunk& ch = vtab[ci++];
        ch.src_off = g.src_off + lo;
        ch.dst_off = dst[k];
        ch.len = int32_t(std::min(kVarintChunk, g.len - lo));
        ch.first_idx = int32_t(before);
        ch.n_values = int32_t(g.ne);
        ch.blob_lo = int32_t(lo);
        before += cc[size_t(q)];
      }
    }
  }
  int32_t* tab = reinterpret_cast<int32_t*>(payload + rt);
  for (int64_t d = 0; d < nd; ++d) {
    const int64_t io = desc[4 * d + 0], wo = desc[4 * d + 1], rows = desc[4 * d + 2], r0 = desc[4 * d + 3];
    if (io & kNarrowFlag) {
      const int64_t ni = io & ~kNarrowFlag;
      const int64_t kind = wo >> kWtsKindShift, w0 = wo & ((int64_t(1) << kWtsKindShift) - 1);
      const int64_t wrow = wts_bytes_per(int(kind)) * wcols;
      for (int64_t r = 0; r < rows; ++r) {
        tab[2 * (r0 + r) + 0] = int32_t(uint32_t(ni + r * idb * fields) | 0x80000000u);
        tab[2 * (r0 + r) + 1] = int32_t(uint32_t(w0 + r * wrow) | uint32_t(kind << kWtsKindShift));
      }
      continue;
    }
    for (int64_t r = 0; r < rows; ++r) {
      tab[2 * (r0 + r) + 0] = int32_t(io + r * 8 * fields);
      tab[2 * (r0 + r) + 1] = int32_t(wo + r * 4 * fields);
    }
  }
  *reinterpret_cast<int32_t*>(base) = int32_t(nd);
  *reinterpret_cast<int64_t*>(base + 8) = row;
  *reinterpret_cast<int64_t*>(base + 16) = rt;
  *reinterpret_cast<int64_t*>(base + 24) = vt;
  *reinterpret_cast<int32_t*>(base + 32) = int32_t(n_chunks);
  *reinterpret_cast<int32_t*>(base + 36) = int32_t(narrow_wcols);
  *reinterpret_cast<int32_t*>(base + 40) = int32_t(idb);
  out.total_rows = row;
  out.n_valid = nd;
  out.n_gpu_varint = int64_t(gjobs.size());
  out.used_bytes = kArenaPayloadOff + vt_end;
  return out;
}

void arena_unpack_cpu(const uint8_t* base, uint8_t* dst, int64_t B, int64_t W, int64_t fields) {
  // the GPU decodes varint ids in its own copy of the arena; do the same here
  arena_varint_cpu(const_cast<uint8_t*>(base));
  // rows through the row table, exactly as the GPU readers find them
  // (csrc/kernels/common.h arena_row): a shared-scatter share carries only its
  // rows' table entries and bytes, not the request descriptors
  int64_t total, rt;
  std::memcpy(&total, base + 8, 8);
  std::memcpy(&rt, base + 16, 8);
  const uint8_t* payload = base + kArenaPayloadOff;
  const int32_t nwc = *reinterpret_cast<const int32_t*>(base + 36);
  const int64_t wcols = nwc > 0 && nwc < fields ? nwc : fields;  // narrowed rows: weights kept per row
  const int64_t idb = *reinterpret_cast<const int32_t*>(base + 40) == 3 ? 3 : 4;  // narrowed rows: bytes per id
  std::memset(dst, 0, size_t(B * W * 8));
  const int64_t n = std::min(total, B);
  for (int64_t row = 0; row < n; ++row) {
    int32_t e[2];
    std::memcpy(e, payload + rt + 8 * row, 8);
    const bool narrow = e[0] < 0;
    const uint8_t* ip = payload + int64_t(uint32_t(e[0]) & 0x7fffffffu);
    const int wkind = narrow ? int(uint32_t(e[1]) >> kWtsKindShift) : kWtsF32;
    const uint8_t* wp = payload + (narrow ? int64_t(uint32_t(e[1]) & ((1u << kWtsKindShift) - 1)) : int64_t(e[1]));
    if (narrow) {  // int32 / 3-byte rows -> int64, weights back to fp32
      for (int64_t f = 0; f < fields; ++f) {
        int32_t id = 0;
        if (idb == 3) {
          id = int32_t(uint32_t(ip[3 * f]) | uint32_t(ip[3 * f + 1]) << 8 | uint32_t(ip[3 * f + 2]) << 16);
        } else {
          std::memcpy(&id, ip + 4 * f, 4);
        }
        const int64_t id64 = id;
        std::memcpy(dst + row * W * 8 + 8 * f, &id64, 8);
      }
      uint8_t* dw = dst + row * W * 8 + 8 * fields;  // dropped columns stay 0
      if (wkind == kWtsF32) {
        std::memcpy(dw, wp, size_t(4 * wcols));
      } else {
        for (int64_t c = 0; c < wcols; ++c) {
          uint32_t v = 0x3f800000u;  // kWtsOnes: 1.0
          if (wkind == kWtsBf16) {
            uint16_t h;
            std::memcpy(&h, wp + 2 * c, 2);
            v = uint32_t(h) << 16;
          }
          std::memcpy(dw + 4 * c, &v, 4);
        }
      }
      continue;
    }
    std::memcpy(dst + row * W * 8, ip, size_t(8 * fields));
    std::memcpy(dst + row * W * 8 + 8 * fields, wp, size_t(4 * fields));
  }
}

}  // namespace runtime
}  // namespace dtfs

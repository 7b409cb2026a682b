// Python bindings for the host-side native runtime: wire codec + batcher.
// Built into distributed_tf_serving_amd/_native*.so by build_ext.py.
#include <torch/extension.h>

#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>

#include "runtime/batcher.h"
#include "runtime/arena.h"
#include "runtime/thread_pool.h"
#include "runtime/trace.h"
#include "wire/tensor_codec.h"
#include "live_bindings.h"
#include "runtime/narrow.h"
#include "net/hpack.h"
#include "runtime/numa.h"
#include "net/h2_client.h"

namespace py = pybind11;
using namespace dtfs;

namespace {

wire::DstType dst_type_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kInt32: return wire::DstType::I32;
    case torch::kInt64: return wire::DstType::I64;
    case torch::kFloat32: return wire::DstType::F32;
    case torch::kBFloat16: return wire::DstType::BF16;
    default: throw py::value_error("decode destination must be int32, int64, float32 or bfloat16");
  }
}

int wire_dtype_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return wire::DT_FLOAT;
    case torch::kFloat64: return wire::DT_DOUBLE;
    case torch::kInt32: return wire::DT_INT32;
    case torch::kInt64: return wire::DT_INT64;
    case torch::kBFloat16: return wire::DT_BFLOAT16;
    case torch::kFloat16: return wire::DT_HALF;
    default: throw py::value_error("unsupported tensor dtype for encoding");
  }
}

// A parsed PredictRequest that keeps its backing bytes alive.
struct ParsedRequest {
  py::bytes holder;
  std::string storage;  // used when constructed from a buffer copy
  wire::PredictRequestView view;

  const wire::TensorView& get(const std::string& key) const {
    const wire::TensorView* t = view.find(key);
    if (!t) throw py::key_error("input '" + key + "' not found in PredictRequest");
    return *t;
  }
};

std::shared_ptr<ParsedRequest> parse_request(py::bytes data) {
  auto r = std::make_shared<ParsedRequest>();
  r->holder = data;
  char* buf;
  Py_ssize_t len;
  if (PyBytes_AsStringAndSize(r->holder.ptr(), &buf, &len) != 0) throw py::error_already_set();
  std::string err;
  bool ok;
  {
    py::gil_scoped_release nogil;
    ok = wire::parse_predict_request(reinterpret_cast<const uint8_t*>(buf), size_t(len), &r->view, &err);
  }
  if (!ok) throw py::value_error("malformed PredictRequest: " + err);
  return r;
}

void decode_into(const ParsedRequest& r, const std::string& key, torch::Tensor dst, int64_t offset,
                 int64_t id_modulo) {
  const wire::TensorView& t = r.get(key);
  if (t.unknown_rank) throw py::value_error("input '" + key + "' has unknown rank");
  if (dst.device().type() != torch::kCPU) throw py::value_error("decode destination must be a CPU tensor");
  const int64_t n = t.num_elements();
  wire::DecodeOpts o;
  o.dst = dst_type_of(dst);
  o.id_modulo = id_modulo;
  char* base;
  if (dst.dim() == 2 && !dst.is_contiguous()) {
    // row view into a packed buffer: offset counts rows; input must be [rows, cols]
    if (dst.stride(1) != 1 || dst.stride(0) < dst.size(1))
      throw py::value_error("decode destination rows must have unit inner stride");
    const int64_t cols = dst.size(1);
    if (t.shape.empty() || t.shape.back() != cols)
      throw py::value_error("input '" + key + "' last dim does not match the destination row width");
    const int64_t rows = n / cols;
    if (offset < 0 || offset + rows > dst.size(0))
      throw py::value_error("decode destination too small for input '" + key + "'");
    o.cols = cols;
    o.ld = dst.stride(0);
    base = static_cast<char*>(dst.data_ptr()) + offset * dst.stride(0) * dst.element_size();
  } else {
    if (!dst.is_contiguous()) throw py::value_error("decode destination must be contiguous or a 2-D row view");
    if (dst.dim() == 2) offset *= dst.size(1);  // 2-D contiguous: offset counts rows
    if (offset < 0 || offset + n > dst.numel())
      throw py::value_error("decode destination too small for input '" + key + "'");
    base = static_cast<char*>(dst.data_ptr()) + offset * dst.element_size();
  }
  std::string err;
  bool ok;
  {
    py::gil_scoped_release nogil;
    ok = wire::decode_into(t, base, n, o, &err);
  }
  if (!ok) throw py::value_error("input '" + key + "': " + err);
}

// A batch of serialized PredictRequests parsed in one GIL-free pass. Rows of
// request i land at rows [row_offset[i], row_offset[i] + rows[i]) of the batch
// destination; malformed requests get rows = 0 and an error string instead of
// failing the batch (the server answers them INVALID_ARGUMENT).
struct ParsedBatch {
  std::vector<py::bytes> holders;
  std::vector<wire::PredictRequestView> views;
  std::vector<const wire::TensorView*> ids_t, wts_t;
  std::vector<int64_t> rows, offsets;
  std::vector<std::string> errors;
  std::string ids_key, wts_key;
  int64_t fields = 0, total_rows = 0;
};

std::shared_ptr<ParsedBatch> parse_batch(const std::vector<py::bytes>& reqs, const std::string& ids_key,
                                         const std::string& wts_key, int64_t fields) {
  auto b = std::make_shared<ParsedBatch>();
  const size_t n = reqs.size();
  b->holders = reqs;
  b->views.resize(n);
  b->ids_t.assign(n, nullptr);
  b->wts_t.assign(n, nullptr);
  b->rows.assign(n, 0);
  b->offsets.assign(n, 0);
  b->errors.assign(n, std::string());
  b->ids_key = ids_key;
  b->wts_key = wts_key;
  b->fields = fields;
  std::vector<std::pair<const char*, size_t>> bufs(n);
  for (size_t i = 0; i < n; ++i) {
    char* p;
    Py_ssize_t len;
    if (PyBytes_AsStringAndSize(b->holders[i].ptr(), &p, &len) != 0) throw py::error_already_set();
    bufs[i] = {p, size_t(len)};
  }
  {
    py::gil_scoped_release nogil;
    int64_t off = 0;
    for (size_t i = 0; i < n; ++i) {
      std::string err;
      auto& v = b->views[i];
      if (!wire::parse_predict_request(reinterpret_cast<const uint8_t*>(bufs[i].first), bufs[i].second, &v, &err)) {
        b->errors[i] = "malformed PredictRequest: " + err;
        continue;
      }
      const wire::TensorView* ti = v.find(ids_key);
      const wire::TensorView* tw = wts_key.empty() ? nullptr : v.find(wts_key);
      if (!ti) {
        b->errors[i] = "input '" + ids_key + "' missing";
        continue;
      }
      if (!wts_key.empty() && !tw) {
        b->errors[i] = "input '" + wts_key + "' missing";
        continue;
      }
      if (ti->unknown_rank || ti->shape.size() != 2 || ti->shape[1] != fields || ti->shape[0] < 0) {
        b->errors[i] = "input '" + ids_key + "' must have shape [B, " + std::to_string(fields) + "]";
        continue;
      }
      if (tw && tw->shape != ti->shape) {
        b->errors[i] = "input '" + wts_key + "' shape differs from '" + ids_key + "'";
        continue;
      }
      const int64_t n_el = ti->num_elements();
      if ((ti->content.n == 0 && ti->num_values > n_el) || (tw && tw->content.n == 0 && tw->num_values > n_el)) {
        b->errors[i] = "more values than the tensor shape holds";
        continue;
      }
      auto content_ok = [n_el](const wire::TensorView* t) {
        return !t || t->content.n == 0 || t->content.n == size_t(n_el) * wire::element_size(t->dtype);
      };
      if (!content_ok(ti) || !content_ok(tw)) {
        b->errors[i] = "tensor_content size does not match shape";
        continue;
      }
      b->ids_t[i] = ti;
      b->wts_t[i] = tw;
      b->rows[i] = ti->shape[0];
      b->offsets[i] = off;
      off += ti->shape[0];
    }
    b->total_rows = off;
  }
  return b;
}

// Decode requests [begin, end) of the batch into row views ids_dst / wts_dst
// (row offset = base_row + offsets[i]). Errors found while decoding are stored
// per request. GIL released throughout: call from several threads on disjoint
// request ranges.
void decode_batch_range(ParsedBatch& b, torch::Tensor ids_dst, c10::optional<torch::Tensor> wts_dst, int64_t begin,
                        int64_t end, int64_t base_row, int64_t id_modulo) {
  auto check_dst = [&](const torch::Tensor& d, const char* what) {
    if (d.device().type() != torch::kCPU || d.dim() != 2 || d.stride(1) != 1 || d.size(1) != b.fields)
      throw py::value_error(std::string(what) + " destination must be a CPU [rows, fields] row view");
    if (base_row < 0 || base_row + b.total_rows > d.size(0))
      throw py::value_error(std::string(what) + " destination has too few rows for the batch");
  };
  check_dst(ids_dst, "ids");
  if (wts_dst) check_dst(*wts_dst, "wts");
  const wire::DstType it = dst_type_of(ids_dst);
  const wire::DstType wt = wts_dst ? dst_type_of(*wts_dst) : wire::DstType::F32;
  char* ibase = static_cast<char*>(ids_dst.data_ptr());
  char* wbase = wts_dst ? static_cast<char*>(wts_dst->data_ptr()) : nullptr;
  const int64_t ild = ids_dst.stride(0), wld = wts_dst ? wts_dst->stride(0) : 0;
  const size_t ies = ids_dst.element_size(), wes = wts_dst ? wts_dst->element_size() : 0;
  begin = std::max<int64_t>(0, begin);
  end = std::min<int64_t>(end, int64_t(b.views.size()));
  py::gil_scoped_release nogil;
  // Work items: a raw (tensor_content) request is split into row chunks so even
  // one large request spreads over the pool; typed-field (varint) requests
  // decode as a whole (their values cannot be addressed by row).
  struct Item {
    int64_t req, r0, r1;
  };
  constexpr int64_t kChunkRows = 128;
  std::vector<Item> items;
  for (int64_t i = begin; i < end; ++i) {
    if (!b.ids_t[i] || b.rows[i] == 0) continue;
    const bool raw = b.ids_t[i]->content.n > 0 && (!b.wts_t[i] || b.wts_t[i]->content.n > 0);
    if (!raw) {
      items.push_back({i, 0, b.rows[i]});
      continue;
    }
    for (int64_t r = 0; r < b.rows[i]; r += kChunkRows) items.push_back({i, r, std::min(b.rows[i], r + kChunkRows)});
  }
  std::vector<std::string> errs(items.size());
  auto sub = [](const wire::TensorView& t, int64_t e0, int64_t e1) {
    wire::TensorView v;  // content-only view of elements [e0, e1)
    v.dtype = t.dtype;
    const size_t es = t.content.n / size_t(std::max<int64_t>(1, t.num_elements()));
    v.content.p = t.content.p + size_t(e0) * es;
    v.content.n = size_t(e1 - e0) * es;
    return v;
  };
  runtime::ThreadPool::global().parallel_for(int64_t(items.size()), [&](int64_t k) {
    const Item& itm = items[k];
    const int64_t i = itm.req;
    const bool whole = itm.r0 == 0 && itm.r1 == b.rows[i];
    const int64_t row = base_row + b.offsets[i] + itm.r0;
    const int64_t e0 = itm.r0 * b.fields, e1 = itm.r1 * b.fields, n = e1 - e0;
    std::string err;
    wire::DecodeOpts o;
    o.dst = it;
    o.id_modulo = id_modulo;
    o.cols = b.fields;
    o.ld = ild;
    const bool ok_ids = whole ? wire::decode_into(*b.ids_t[i], ibase + size_t(row * ild) * ies, n, o, &err)
                              : wire::decode_into(sub(*b.ids_t[i], e0, e1), ibase + size_t(row * ild) * ies, n, o, &err);
    if (!ok_ids) {
      errs[k] = "input '" + b.ids_key + "': " + err;
      return;
    }
    if (wbase && b.wts_t[i]) {
      wire::DecodeOpts ow;
      ow.dst = wt;
      ow.cols = b.fields;
      ow.ld = wld;
      const bool ok = whole ? wire::decode_into(*b.wts_t[i], wbase + size_t(row * wld) * wes, n, ow, &err)
                            : wire::decode_into(sub(*b.wts_t[i], e0, e1), wbase + size_t(row * wld) * wes, n, ow, &err);
      if (!ok) errs[k] = "input '" + b.wts_key + "': " + err;
    }
  });
  for (size_t k = 0; k < items.size(); ++k)
    if (!errs[k].empty() && b.errors[items[k].req].empty()) b.errors[items[k].req] = errs[k];
}

// ---------------------------------------------------------------- request arena
// Thin wrappers over csrc/runtime/arena.cpp (layout documented there).
using runtime::ArenaBatch;
using runtime::kArenaMaxRequests;
using runtime::kArenaPayloadOff;

void check_arena(const torch::Tensor& arena) {
  if (arena.device().type() != torch::kCPU || !arena.is_contiguous() || arena.scalar_type() != torch::kUInt8)
    throw py::value_error("arena must be a contiguous CPU uint8 tensor");
}

// Copy serialized requests into the arena payload (parallel memcpy, GIL-free);
// returns their (offset, length) spans relative to the payload start.
std::vector<std::pair<int64_t, int64_t>> arena_place(torch::Tensor arena, const std::vector<py::bytes>& reqs,
                                                     int64_t start) {
  check_arena(arena);
  std::vector<std::pair<const char*, size_t>> src(reqs.size());
  for (size_t i = 0; i < reqs.size(); ++i) {
    char* p;
    Py_ssize_t len;
    if (PyBytes_AsStringAndSize(reqs[i].ptr(), &p, &len) != 0) throw py::error_already_set();
    src[i] = {p, size_t(len)};
  }
  py::gil_scoped_release nogil;
  try {
    return runtime::arena_place(arena.data_ptr<uint8_t>(), arena.numel(), src, start);
  } catch (const std::invalid_argument& e) {
    py::gil_scoped_acquire g;
    throw py::value_error(e.what());
  }
}

ArenaBatch arena_build(torch::Tensor arena, const std::vector<std::pair<int64_t, int64_t>>& spans,
                       const std::string& ids_key, const std::string& wts_key, int64_t fields, int64_t max_rows,
                       int64_t varint_chunks) {
  check_arena(arena);
  py::gil_scoped_release nogil;
  try {
    return runtime::arena_build(arena.data_ptr<uint8_t>(), arena.numel(), spans, ids_key, wts_key, fields, max_rows,
                                varint_chunks);
  } catch (const std::invalid_argument& e) {
    py::gil_scoped_acquire g;
    throw py::value_error(e.what());
  }
}

// Host reference of the GPU unpack (tests, CPU serving): arena -> packed rows.
void arena_unpack_cpu(torch::Tensor arena, torch::Tensor packed, int64_t fields) {
  check_arena(arena);
  if (packed.scalar_type() != torch::kInt64 || packed.dim() != 2 || !packed.is_contiguous())
    throw py::value_error("packed must be a contiguous int64 [B, W] tensor");
  if (packed.size(1) * 8 < 12 * fields) throw py::value_error("packed rows too narrow for the field count");
  const uint8_t* base = arena.data_ptr<uint8_t>();
  uint8_t* dst = reinterpret_cast<uint8_t*>(packed.data_ptr<int64_t>());
  const int64_t W = packed.size(1), B = packed.size(0);
  py::gil_scoped_release nogil;
  runtime::arena_unpack_cpu(base, dst, B, W, fields);
}

// One PredictResponse per request: outputs[key] = scores[offsets[i] : +rows[i]]
// as float_val (what the reference client reads, DCNClient.java:162).
std::vector<py::bytes> encode_batch_responses(const std::string& name, const std::string& sig, py::object version,
                                              const std::string& key, torch::Tensor scores,
                                              const std::vector<int64_t>& rows, const std::vector<int64_t>& offsets,
                                              bool raw) {
  if (scores.device().type() != torch::kCPU || scores.scalar_type() != torch::kFloat32 || !scores.is_contiguous())
    throw py::value_error("scores must be a contiguous CPU fp32 tensor");
  if (rows.size() != offsets.size()) throw py::value_error("rows/offsets length mismatch");
  wire::ModelSpecOut spec;
  spec.name = name;
  spec.signature_name = sig;
  if (!version.is_none()) {
    spec.has_version = true;
    spec.version = version.cast<int64_t>();
  }
  const float* s = scores.data_ptr<float>();
  const int64_t ns = scores.numel();
  std::vector<std::string> outs(rows.size());
  {
    py::gil_scoped_release nogil;
    for (size_t i = 0; i < rows.size(); ++i) {
      if (offsets[i] < 0 || rows[i] < 0 || offsets[i] + rows[i] > ns) continue;
      wire::TensorOut t;
      t.key = key;
      t.dtype = wire::DT_FLOAT;
      t.shape = {rows[i]};
      t.data = s + offsets[i];
      t.n = rows[i];
      t.raw = raw;
      outs[i] = wire::encode_predict_response(spec, {t});
    }
  }
  std::vector<py::bytes> res;
  res.reserve(outs.size());
  for (auto& o : outs) res.emplace_back(o);
  return res;
}

std::vector<wire::TensorOut> tensors_out(const std::vector<std::pair<std::string, torch::Tensor>>& items,
                                         bool raw, std::vector<torch::Tensor>* keep) {
  std::vector<wire::TensorOut> outs;
  for (const auto& kv : items) {
    torch::Tensor t = kv.second.contiguous().cpu();
    keep->push_back(t);
    wire::TensorOut o;
    o.key = kv.first;
    o.dtype = wire_dtype_of(t);
    for (int64_t d : t.sizes()) o.shape.push_back(d);
    o.data = t.data_ptr();
    o.n = t.numel();
    o.raw = raw || !(o.dtype == wire::DT_FLOAT || o.dtype == wire::DT_INT64 || o.dtype == wire::DT_INT32 ||
                     o.dtype == wire::DT_DOUBLE);
    outs.push_back(std::move(o));
  }
  return outs;
}

wire::ModelSpecOut spec_of(const std::string& name, const std::string& sig, py::object version) {
  wire::ModelSpecOut s;
  s.name = name;
  s.signature_name = sig;
  if (!version.is_none()) {
    s.has_version = true;
    s.version = version.cast<int64_t>();
  }
  return s;
}

// ---------------------------------------------------------------- live server (CPU backend)
// The device side of a CPU live server is a Python callable
// forward(arena_index, slot, bucket_index) that scores the parsed arena into
// scores[slot][bucket_index] (serving/live.py: FanoutEngine.launch on CPU).
// Used for BASELINE config 1 (Wide&Deep-tiny on a CPU backend) and to test the
// batching core without a GPU.
class PyCpuBackend : public runtime::StepBackend {
 public:
  PyCpuBackend(std::vector<int64_t> buckets, std::vector<std::vector<torch::Tensor>> scores,
               std::vector<const uint8_t*> arenas, py::function fwd)
      : buckets_(std::move(buckets)), arenas_(std::move(arenas)), fwd_(std::move(fwd)) {
    TORCH_CHECK(!scores.empty(), "need at least one slot");
    for (auto& per_slot : scores) {
      TORCH_CHECK(per_slot.size() == buckets_.size(), "scores: one tensor per bucket per slot");
      std::vector<std::pair<const float*, int64_t>> v;
      for (size_t b = 0; b < per_slot.size(); ++b) {
        const auto& t = per_slot[b];
        TORCH_CHECK(t.device().is_cpu() && t.is_contiguous() && t.scalar_type() == torch::kFloat32,
                    "scores must be contiguous CPU fp32 tensors");
        v.emplace_back(t.data_ptr<float>(), t.numel());
      }
      scores_.push_back(std::move(v));
    }
    err_.assign(scores_.size(), std::string());
  }
  ~PyCpuBackend() override {
    py::gil_scoped_acquire g;
    fwd_ = py::function();
  }
  int slots() const override { return int(scores_.size()); }
  const std::vector<int64_t>& buckets() const override { return buckets_; }
  void launch(int slot, int b, const uint8_t* arena, const runtime::ArenaBatch&) override {
    const auto it = std::find(arenas_.begin(), arenas_.end(), arena);
    if (it == arenas_.end()) throw std::runtime_error("unknown arena");
    py::gil_scoped_acquire g;
    try {
      fwd_(int(it - arenas_.begin()), slot, b);
      err_[size_t(slot)].clear();
    } catch (py::error_already_set& e) {
      err_[size_t(slot)] = e.what();  // reported by wait(): the step failed
    }
  }
  bool wait(int slot, int64_t, std::string* err) override {
    if (err_[size_t(slot)].empty()) return true;
    *err = err_[size_t(slot)];
    return false;
  }
  const float* scores(int slot, int b) const override { return scores_[size_t(slot)][size_t(b)].first; }
  int64_t scores_len(int slot, int b) const override { return scores_[size_t(slot)][size_t(b)].second; }

 private:
  std::vector<int64_t> buckets_;
  std::vector<std::vector<std::pair<const float*, int64_t>>> scores_;
  std::vector<const uint8_t*> arenas_;
  py::function fwd_;
  std::vector<std::string> err_;
};

struct PyCpuLive {
  std::vector<py::object> keep;
  std::unique_ptr<PyCpuBackend> backend;
  std::unique_ptr<runtime::LiveServer> srv;
  ~PyCpuLive() {
    py::gil_scoped_release nogil;  // the server threads may need the GIL to finish
    srv.reset();
  }
};

PyCpuLive* make_cpu_live(py::dict cfg, std::vector<int64_t> buckets, py::list scores, py::list arenas,
                         py::function fwd, py::object control) {
  auto* p = new PyCpuLive();
  runtime::StepControl* ctl = dtfs_live::control_from(control, &p->keep);
  auto ar = dtfs_live::arenas_from(arenas, false, &p->keep);
  std::vector<const uint8_t*> bases;
  for (auto& a : ar) bases.push_back(a.first);
  std::vector<std::vector<torch::Tensor>> sc;
  for (auto per_slot : scores) {
    std::vector<torch::Tensor> v;
    for (auto t : per_slot.cast<py::list>()) v.push_back(t.cast<torch::Tensor>());
    sc.push_back(std::move(v));
  }
  p->keep.push_back(scores);
  p->backend = std::make_unique<PyCpuBackend>(std::move(buckets), std::move(sc), std::move(bases), fwd);
  p->srv = std::make_unique<runtime::LiveServer>(p->backend.get(), dtfs_live::live_config_from(cfg), std::move(ar),
                                                 ctl);
  return p;
}

}  // namespace

// Known-answer checks of the HPACK pieces the native front door uses
// (tests/test_native_front.py); vectors from RFC 7541 Appendix C.
py::dict hpack_selftest() {
  namespace n = dtfs::net;
  py::dict o;
  bool rt = true;
  std::string all;
  for (int c = 0; c < 256; ++c) all.push_back(char(c));
  for (const std::string& s : {all, std::string("application/grpc"), std::string("grpc-java-netty/1.12.0"),
                               std::string(""), std::string("te"), std::string(300, '~')}) {
    std::string d;
    const std::string e = n::huffman_encode(s);
    rt = rt && n::huffman_decode(reinterpret_cast<const uint8_t*>(e.data()), e.size(), &d) && d == s;
  }
  // C.4.1: "www.example.com" -> f1e3 c2e5 f23a 6ba0 ab90 f4ff; C.4.2: "no-cache" -> a8eb 1064 9cbf
  rt = rt && n::huffman_encode("www.example.com") == std::string("\xf1\xe3\xc2\xe5\xf2\x3a\x6b\xa0\xab\x90\xf4\xff", 12);
  rt = rt && n::huffman_encode("no-cache") == std::string("\xa8\xeb\x10\x64\x9c\xbf", 6);
  o["huffman_roundtrip"] = rt;
  // C.4.1 request: :method GET, :scheme http, :path /, :authority www.example.com (Huffman, incremental indexing)
  const std::string c41("\x82\x86\x84\x41\x8c\xf1\xe3\xc2\xe5\xf2\x3a\x6b\xa0\xab\x90\xf4\xff", 17);
  n::HpackDecoder dec;
  std::vector<n::Header> hs;
  std::string err;
  bool ok = dec.decode(reinterpret_cast<const uint8_t*>(c41.data()), c41.size(), &hs, &err) && hs.size() == 4 &&
            hs[0] == n::Header(":method", "GET") && hs[1] == n::Header(":scheme", "http") &&
            hs[2] == n::Header(":path", "/") && hs[3] == n::Header(":authority", "www.example.com");
  o["static_decode"] = ok;
  // C.4.2: the same connection's next block refers to dynamic entry 62 (:authority) and adds cache-control
  const std::string c42("\x82\x86\x84\xbe\x58\x86\xa8\xeb\x10\x64\x9c\xbf", 12);
  hs.clear();
  ok = dec.decode(reinterpret_cast<const uint8_t*>(c42.data()), c42.size(), &hs, &err) && hs.size() == 5 &&
       hs[3] == n::Header(":authority", "www.example.com") && hs[4] == n::Header("cache-control", "no-cache") &&
       dec.table_entries() == 2 && dec.table_size() == 110;
  o["dynamic_table"] = ok;
  // padding that is not a prefix of EOS, and 8+ bits of padding, are errors
  std::string d;
  const uint8_t bad1[] = {0x00};        // '0' (00000) + padding 000: zeros
  const uint8_t bad2[] = {0x1f, 0xff};  // 'a' (00011) + 11 one-bits of padding
  o["bad_padding_rejected"] = !n::huffman_decode(bad1, 1, &d) && !n::huffman_decode(bad2, 2, &d);
  py::list ts;
  for (const char* t : {"1S", "250m", "100u", "1000n", "2H", "x"}) ts.append(n::parse_grpc_timeout(t));
  o["timeouts"] = ts;
  o["percent"] = n::grpc_percent_encode("a%b\nc\xc3\xa9");
  return o;
}

PYBIND11_MODULE(_native, m) {
  // NUMA placement (runtime/numa.h; utils/affinity.py)
  m.def("numa_node_count", &dtfs::runtime::numa_node_count);
  m.def("numa_node_cpus", &dtfs::runtime::numa_node_cpus, py::arg("node"));
  m.def("pci_numa_node", &dtfs::runtime::pci_numa_node, py::arg("bus_id"));
  m.def("bind_process_cpus", &dtfs::runtime::bind_process_cpus, py::arg("cpus"),
        "bind every thread of this process to these CPUs; returns the threads re-bound");
  m.def("prefer_numa_node", &dtfs::runtime::prefer_numa_node, py::arg("node"));
  m.def(
      "alloc_on_node",
      [](int64_t bytes, int node) {
        void* p = dtfs::runtime::alloc_on_node(size_t(bytes), node);
        const size_t n = size_t(bytes);
        return torch::from_blob(p, {bytes}, [n](void* q) { dtfs::runtime::free_on_node(q, n); },
                                torch::TensorOptions().dtype(torch::kUInt8));
      },
      py::arg("bytes"), py::arg("node"), "uint8 CPU tensor whose pages live on `node` (mmap + mbind + touch)");
  m.def(
      "page_numa_node", [](const torch::Tensor& t, int64_t offset) {
        return dtfs::runtime::page_numa_node(static_cast<const uint8_t*>(t.data_ptr()) + offset);
      },
      py::arg("tensor"), py::arg("offset") = 0);
  m.def("hpack_selftest", &hpack_selftest, "HPACK known-answer checks (RFC 7541 Appendix C)");
  m.def(
      "grpc_call",
      [](const std::string& host, int port, const std::string& path, py::bytes data, double timeout_s) {
        const std::string req = data;
        int st = -1;
        std::string msg, body;
        bool ok;
        {
          py::gil_scoped_release nogil;
          dtfs::net::H2Client c(host, port);
          ok = c.call(path, req, timeout_s > 0 ? int64_t(timeout_s * 1e6) : 0, &st, &msg, &body);
        }
        if (!ok) throw std::runtime_error("gRPC transport failure: " + msg);
        return py::make_tuple(st, msg, py::bytes(body));
      },
      py::arg("host"), py::arg("port"), py::arg("path"), py::arg("request"), py::arg("timeout_s") = 0.0,
      "One unary gRPC call over the native h2c client: (status, message, response bytes).");
  m.def(
      "run_grpc_load",
      [](const std::string& host, int port, const std::string& path, const std::vector<std::string>& requests,
         int concurrency, int64_t warmup, int64_t count, double timeout_s) {
        dtfs::net::GrpcLoadSpec sp;
        sp.concurrency = concurrency;
        sp.warmup = warmup;
        sp.count = count;
        sp.timeout_us = timeout_s > 0 ? int64_t(timeout_s * 1e6) : 0;
        dtfs::net::GrpcLoadResult r;
        {
          py::gil_scoped_release nogil;
          r = dtfs::net::run_grpc_load(host, port, path, requests, sp);
        }
        py::dict o;
        o["latency_us"] = r.latency_us;
        o["ok"] = r.ok;
        o["errors"] = r.errors;
        o["window_us"] = r.window_us;
        o["wall_us"] = r.wall_us;
        o["first_error"] = r.first_error;
        return o;
      },
      py::arg("host"), py::arg("port"), py::arg("path"), py::arg("requests"), py::arg("concurrency") = 6,
      py::arg("warmup") = 0, py::arg("count") = 1000, py::arg("timeout_s") = 0.0,
      "Closed-loop gRPC load over native h2c clients (one connection per client thread).");
  m.doc() = "distributed_tf_serving_amd host runtime: zero-copy TF-Serving wire codec + dynamic batcher";

  py::class_<ParsedRequest, std::shared_ptr<ParsedRequest>>(m, "ParsedPredictRequest")
      .def_property_readonly("model_name", [](const ParsedRequest& r) { return r.view.model_name; })
      .def_property_readonly("signature_name", [](const ParsedRequest& r) { return r.view.signature_name; })
      .def_property_readonly("version", [](const ParsedRequest& r) -> py::object {
        if (!r.view.has_version) return py::none();
        return py::int_(r.view.version);
      })
      .def_property_readonly("output_filter", [](const ParsedRequest& r) { return r.view.output_filter; })
      .def("input_names", [](const ParsedRequest& r) {
        std::vector<std::string> k;
        for (const auto& kv : r.view.inputs) k.push_back(kv.first);
        return k;
      })
      .def("has_input", [](const ParsedRequest& r, const std::string& k) { return r.view.find(k) != nullptr; })
      .def("shape", [](const ParsedRequest& r, const std::string& k) { return r.get(k).shape; })
      .def("dtype", [](const ParsedRequest& r, const std::string& k) { return r.get(k).dtype; })
      .def("num_elements", [](const ParsedRequest& r, const std::string& k) { return r.get(k).num_elements(); })
      .def("num_values", [](const ParsedRequest& r, const std::string& k) {
        const auto& t = r.get(k);
        return t.content.n ? t.num_elements() : t.num_values;
      })
      .def("is_raw", [](const ParsedRequest& r, const std::string& k) { return r.get(k).content.n > 0; })
      .def("decode_into", &decode_into, py::arg("key"), py::arg("dst"), py::arg("offset") = 0,
           py::arg("id_modulo") = 0,
           "Decode input `key` (TF fill semantics) into dst[offset: offset+numel], narrowing dtypes.");

  m.def("parse_predict_request", &parse_request, py::arg("data"));

  py::class_<ParsedBatch, std::shared_ptr<ParsedBatch>>(m, "ParsedBatch")
      .def_readonly("rows", &ParsedBatch::rows)
      .def_readonly("offsets", &ParsedBatch::offsets)
      .def_readonly("errors", &ParsedBatch::errors)
      .def_readonly("total_rows", &ParsedBatch::total_rows)
      .def_readonly("fields", &ParsedBatch::fields)
      .def("__len__", [](const ParsedBatch& b) { return b.views.size(); })
      .def("model_name", [](const ParsedBatch& b, size_t i) { return b.views.at(i).model_name; })
      .def("signature_name", [](const ParsedBatch& b, size_t i) { return b.views.at(i).signature_name; })
      .def("version", [](const ParsedBatch& b, size_t i) -> py::object {
        const auto& v = b.views.at(i);
        return v.has_version ? py::object(py::int_(v.version)) : py::object(py::none());
      })
      .def("output_filter", [](const ParsedBatch& b, size_t i) { return b.views.at(i).output_filter; })
      .def("decode", &decode_batch_range, py::arg("ids_dst"), py::arg("wts_dst"), py::arg("begin") = 0,
           py::arg("end") = int64_t(1) << 62, py::arg("base_row") = 0, py::arg("id_modulo") = 0);

  py::class_<ArenaBatch>(m, "ArenaBatch")
      .def_readonly("rows", &ArenaBatch::rows)
      .def_readonly("offsets", &ArenaBatch::offsets)
      .def_readonly("errors", &ArenaBatch::errors)
      .def_readonly("total_rows", &ArenaBatch::total_rows)
      .def_readonly("used_bytes", &ArenaBatch::used_bytes)
      .def_readonly("n_valid", &ArenaBatch::n_valid)
      .def_readonly("n_decoded", &ArenaBatch::n_decoded)
      .def_readonly("n_gpu_varint", &ArenaBatch::n_gpu_varint);
  m.attr("ARENA_PAYLOAD_OFF") = kArenaPayloadOff;
  m.attr("ARENA_MAX_REQUESTS") = kArenaMaxRequests;
  m.def("arena_place", &arena_place, py::arg("arena"), py::arg("requests"), py::arg("start") = 0);
  m.def("arena_build", &arena_build, py::arg("arena"), py::arg("spans"), py::arg("ids_key") = "feat_ids",
        py::arg("wts_key") = "feat_wts", py::arg("fields") = 43, py::arg("max_rows") = int64_t(1) << 40,
        py::arg("varint_chunks") = 0);
  m.def("arena_varint_capacity", &runtime::arena_varint_capacity, py::arg("max_rows"), py::arg("fields"),
        py::arg("max_requests") = runtime::kArenaMaxRequests);
  m.def("arena_unpack_cpu", &arena_unpack_cpu, py::arg("arena"), py::arg("packed"), py::arg("fields"));

  m.def("parse_batch", &parse_batch, py::arg("requests"), py::arg("ids_key") = "feat_ids",
        py::arg("wts_key") = "feat_wts", py::arg("fields") = 43,
        "Parse many serialized PredictRequests (GIL released); see ParsedBatch.decode.");
  m.def("encode_batch_responses", &encode_batch_responses, py::arg("model_name"), py::arg("signature_name"),
        py::arg("version"), py::arg("key"), py::arg("scores"), py::arg("rows"), py::arg("offsets"),
        py::arg("raw") = false);

  m.def(
      "encode_predict_response",
      [](const std::string& name, const std::string& sig, py::object version,
         const std::vector<std::pair<std::string, torch::Tensor>>& outputs, bool raw) {
        std::vector<torch::Tensor> keep;
        auto outs = tensors_out(outputs, raw, &keep);
        auto spec = spec_of(name, sig, version);
        std::string s;
        {
          py::gil_scoped_release nogil;
          s = wire::encode_predict_response(spec, outs);
        }
        return py::bytes(s);
      },
      py::arg("model_name"), py::arg("signature_name"), py::arg("version"), py::arg("outputs"),
      py::arg("raw") = false);

  m.def(
      "encode_predict_request",
      [](const std::string& name, const std::string& sig, py::object version,
         const std::vector<std::pair<std::string, torch::Tensor>>& inputs, bool raw,
         const std::vector<std::string>& output_filter) {
        std::vector<torch::Tensor> keep;
        auto ins = tensors_out(inputs, raw, &keep);
        auto spec = spec_of(name, sig, version);
        std::string s;
        {
          py::gil_scoped_release nogil;
          s = wire::encode_predict_request(spec, ins, output_filter);
        }
        return py::bytes(s);
      },
      py::arg("model_name"), py::arg("signature_name"), py::arg("version"), py::arg("inputs"),
      py::arg("raw") = false, py::arg("output_filter") = std::vector<std::string>{});

  m.def("f32_to_bf16_bits", [](float f) { return wire::f32_to_bf16(f); });

  py::class_<runtime::BatchItem>(m, "BatchItem")
      .def_readonly("ticket", &runtime::BatchItem::ticket)
      .def_readonly("rows", &runtime::BatchItem::rows)
      .def_readonly("enqueue_us", &runtime::BatchItem::enqueue_us)
      .def_readonly("deadline_us", &runtime::BatchItem::deadline_us);

  py::class_<runtime::Batch>(m, "Batch")
      .def_readonly("items", &runtime::Batch::items)
      .def_readonly("expired", &runtime::Batch::expired)
      .def_readonly("rows", &runtime::Batch::rows)
      .def_readonly("closed", &runtime::Batch::closed);

  py::class_<runtime::BatcherStats>(m, "BatcherStats")
      .def_readonly("submitted", &runtime::BatcherStats::submitted)
      .def_readonly("rejected", &runtime::BatcherStats::rejected)
      .def_readonly("batches", &runtime::BatcherStats::batches)
      .def_readonly("batched_rows", &runtime::BatcherStats::batched_rows)
      .def_readonly("expired", &runtime::BatcherStats::expired)
      .def_readonly("full_batches", &runtime::BatcherStats::full_batches)
      .def_readonly("timeout_batches", &runtime::BatcherStats::timeout_batches);

  py::class_<runtime::DynamicBatcher>(m, "DynamicBatcher")
      .def(py::init<int64_t, int64_t, int64_t>(), py::arg("max_batch_rows"), py::arg("batch_timeout_us"),
           py::arg("max_queued_rows") = 0)
      .def("submit", &runtime::DynamicBatcher::submit, py::arg("ticket"), py::arg("rows"),
           py::arg("deadline_us") = 0)
      .def("next_batch", &runtime::DynamicBatcher::next_batch, py::arg("wait_us") = -1, py::arg("eager") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("close", &runtime::DynamicBatcher::close)
      .def_property_readonly("closed", &runtime::DynamicBatcher::closed)
      .def_property_readonly("queued_rows", &runtime::DynamicBatcher::queued_rows)
      .def_property_readonly("max_batch_rows", &runtime::DynamicBatcher::max_batch_rows)
      .def_property_readonly("batch_timeout_us", &runtime::DynamicBatcher::batch_timeout_us)
      .def("stats", &runtime::DynamicBatcher::stats);

  {
    py::class_<PyCpuLive> c(m, "LiveServer",
                            "Live serving core (csrc/runtime/live_server.h) with a CPU backend: a Python "
                            "forward(arena_index, slot, bucket_index) scores each batch");
    c.def(py::init(&make_cpu_live), py::arg("config"), py::arg("buckets"), py::arg("scores"), py::arg("arenas"),
          py::arg("forward"), py::arg("control") = py::none());
    dtfs_live::def_live_methods(c);
  }
  dtfs_live::def_step_control(m);
  dtfs_live::def_shared_scatter(m);
  dtfs_live::def_grpc_front<PyCpuLive>(m);
  m.attr("STATUS_OVERSIZE") = int(runtime::kOversize);
  m.attr("STATUS_CALLER_PATH") = int(runtime::kCallerPath);
  m.def(
      "narrow_ids",
      [](torch::Tensor ids, int64_t modulo) {
        TORCH_CHECK(ids.device().is_cpu() && ids.scalar_type() == torch::kInt64, "ids must be CPU int64");
        TORCH_CHECK(modulo >= 1 && modulo < (int64_t(1) << 31), "modulo must be in [1, 2^31)");
        auto src = ids.contiguous();
        auto out = torch::empty(src.sizes(), torch::kInt32);
        runtime::narrow_ids(reinterpret_cast<const uint8_t*>(src.data_ptr()), out.data_ptr<int32_t>(), src.numel(),
                            modulo);
        return out;
      },
      py::arg("ids"), py::arg("modulo"), "Host K0: int64 ids -> int32 rows (python-style id mod modulo).");
  m.def(
      "narrow_ids24",
      [](torch::Tensor ids, int64_t modulo) {
        TORCH_CHECK(ids.device().is_cpu() && ids.scalar_type() == torch::kInt64, "ids must be CPU int64");
        TORCH_CHECK(modulo >= 1 && modulo <= (int64_t(1) << 24), "modulo must be in [1, 2^24]");
        auto src = ids.contiguous();
        auto out = torch::empty({3 * src.numel() + runtime::kNarrow24Slack}, torch::kUInt8);
        runtime::narrow_ids24(reinterpret_cast<const uint8_t*>(src.data_ptr()), out.data_ptr<uint8_t>(), src.numel(),
                              modulo);
        return out.narrow(0, 0, 3 * src.numel());
      },
      py::arg("ids"), py::arg("modulo"), "Host K0: int64 ids -> 3-byte little-endian rows (id mod modulo <= 2^24).");
  m.def(
      "classify_weights",
      [](torch::Tensor wts, int64_t wcols) {
        TORCH_CHECK(wts.device().is_cpu() && wts.scalar_type() == torch::kFloat32 && wts.dim() == 2,
                    "wts must be CPU fp32 [rows, fields]");
        TORCH_CHECK(wcols >= 1 && wcols <= wts.size(1), "wcols must be in [1, fields]");
        auto src = wts.contiguous();
        return runtime::classify_weights(reinterpret_cast<const uint8_t*>(src.data_ptr()), src.size(0), src.size(1),
                                         wcols);
      },
      py::arg("wts"), py::arg("wcols"),
      "Host K0: the cheapest exact form of a request's first wcols weights per row (0 fp32, 1 bf16, 2 all 1.0).");
  m.def("now_us", &runtime::now_us);
  m.def("trace_enabled", &trace::enabled);
  m.def("trace_push", [](const std::string& s) { trace::push(s.c_str()); }, py::arg("name"));
  m.def("trace_pop", &trace::pop);
  m.def("trace_mark", [](const std::string& s) { trace::mark(s.c_str()); }, py::arg("name"));
}

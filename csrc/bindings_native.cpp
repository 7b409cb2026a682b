// Python bindings for the host-side native runtime: wire codec + batcher.
// Built into distributed_tf_serving_amd/_native*.so by build_ext.py.
#include <torch/extension.h>

#include <pybind11/stl.h>

#include "runtime/batcher.h"
#include "wire/tensor_codec.h"

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
  if (!dst.is_contiguous() || dst.device().type() != torch::kCPU)
    throw py::value_error("decode destination must be a contiguous CPU tensor");
  const int64_t n = t.num_elements();
  if (offset < 0 || offset + n > dst.numel())
    throw py::value_error("decode destination too small for input '" + key + "'");
  wire::DecodeOpts o;
  o.dst = dst_type_of(dst);
  o.id_modulo = id_modulo;
  char* base = static_cast<char*>(dst.data_ptr()) + offset * dst.element_size();
  std::string err;
  bool ok;
  {
    py::gil_scoped_release nogil;
    ok = wire::decode_into(t, base, n, o, &err);
  }
  if (!ok) throw py::value_error("input '" + key + "': " + err);
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

}  // namespace

PYBIND11_MODULE(_native, m) {
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
      .def("next_batch", &runtime::DynamicBatcher::next_batch, py::arg("wait_us") = -1,
           py::call_guard<py::gil_scoped_release>())
      .def("close", &runtime::DynamicBatcher::close)
      .def_property_readonly("closed", &runtime::DynamicBatcher::closed)
      .def_property_readonly("queued_rows", &runtime::DynamicBatcher::queued_rows)
      .def_property_readonly("max_batch_rows", &runtime::DynamicBatcher::max_batch_rows)
      .def_property_readonly("batch_timeout_us", &runtime::DynamicBatcher::batch_timeout_us)
      .def("stats", &runtime::DynamicBatcher::stats);

  m.def("now_us", &runtime::now_us);
}

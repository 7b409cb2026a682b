// Zero-copy protobuf codec for the TF-Serving Predict hot path.
//
// There are no C++ protobuf headers in this image, and the generic protobuf
// runtime is exactly what the reference pays for on its hot loop (boxed Long /
// Float lists -> varint packing, reference DCNClient.java:98-108, and the
// mirror-image parse on the server). This codec walks the wire format once,
// records spans into the caller's buffer, and decodes tensor payloads straight
// into a destination buffer (typically pinned host memory that is then DMA'd to
// the GPU), narrowing dtypes on the fly (int64 ids -> int32 row ids with an
// optional modulo, fp32 weights -> fp32/bf16).
//
// Wire schema (field numbers): distributed_tf_serving_amd/wire/protos/*.proto,
// identical to reference predict.proto:12-40 and tensor.proto:14-84.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace dtfs {
namespace wire {

// tensorflow.DataType values used by the codec (reference types.proto:11-67).
enum DType : int {
  DT_INVALID = 0,
  DT_FLOAT = 1,
  DT_DOUBLE = 2,
  DT_INT32 = 3,
  DT_UINT8 = 4,
  DT_INT16 = 5,
  DT_INT8 = 6,
  DT_STRING = 7,
  DT_INT64 = 9,
  DT_BOOL = 10,
  DT_BFLOAT16 = 14,
  DT_UINT16 = 17,
  DT_HALF = 19,
  DT_UINT32 = 22,
  DT_UINT64 = 23,
};

// Destination element types for decode_into().
enum class DstType : int { I32 = 0, I64 = 1, F32 = 2, BF16 = 3 };

struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
};

// One TensorProto, as spans into the request buffer.
struct TensorView {
  int dtype = DT_INVALID;
  std::vector<int64_t> shape;
  bool unknown_rank = false;
  Span content;                    // tensor_content (field 4)
  int value_field = 0;             // typed field number the values came from
  bool value_packed_varint = false;
  bool value_fixed32 = false;
  bool value_fixed64 = false;
  std::vector<Span> packed;        // packed chunks of the typed field
  std::vector<uint64_t> unpacked;  // raw bits of non-packed typed values
  int64_t num_values = 0;          // typed values present (not counting fill)

  int64_t num_elements() const;
};

struct PredictRequestView {
  std::string model_name;
  std::string signature_name;
  bool has_version = false;
  int64_t version = 0;
  std::vector<std::string> output_filter;
  std::vector<std::pair<std::string, TensorView>> inputs;

  const TensorView* find(const std::string& key) const;
};

// Parse a serialized tensorflow.serving.PredictRequest. Returns false and sets
// *err on malformed input. The view keeps pointers into [buf, buf+len).
// count_packed_varints = false leaves num_values = -1 for packed varint
// fields (the caller counts them itself, e.g. the arena build, which counts
// per GPU decode chunk anyway).
bool parse_predict_request(const uint8_t* buf, size_t len, PredictRequestView* out, std::string* err,
                           bool count_packed_varints = true);

// Terminator bytes (MSB clear) = complete varints in [p, p + n); AVX2 when
// the CPU has it.
int64_t count_varint_terminators(const uint8_t* p, size_t n);

// Bytes per element of a TF DataType in tensor_content (0: unsupported).
size_t element_size(int dtype);

// Parse one serialized TensorProto.
bool parse_tensor(const uint8_t* buf, size_t len, TensorView* out, std::string* err);

struct DecodeOpts {
  DstType dst = DstType::F32;
  int64_t id_modulo = 0;  // >0: ids become ((id % m) + m) % m (hash into table rows)
  int64_t cols = 0;       // destination row view: elements per row (0: contiguous)
  int64_t ld = 0;         // elements between row starts (0 or == cols: contiguous)
};

// Decode the tensor's elements (with TF fill semantics) into dst, which must
// hold num_elements() elements of opts.dst. Returns false on dtype mismatch or
// too many values.
bool decode_into(const TensorView& t, void* dst, int64_t n_elems, const DecodeOpts& opts, std::string* err);

// ---- encoders ------------------------------------------------------------
struct ModelSpecOut {
  std::string name;
  std::string signature_name;
  bool has_version = false;
  int64_t version = 0;
};

struct TensorOut {
  std::string key;
  int dtype = DT_FLOAT;          // DT_FLOAT, DT_INT64, DT_INT32, DT_DOUBLE
  std::vector<int64_t> shape;
  const void* data = nullptr;    // host array of dtype
  int64_t n = 0;
  bool raw = false;              // tensor_content instead of the typed field
};

// Serialize a PredictResponse (outputs map + model_spec), fields in number
// order as protobuf's own serializer emits them.
std::string encode_predict_response(const ModelSpecOut& spec, const std::vector<TensorOut>& outputs);

// Serialize a PredictRequest (model_spec, inputs map, output_filter).
std::string encode_predict_request(const ModelSpecOut& spec, const std::vector<TensorOut>& inputs,
                                   const std::vector<std::string>& output_filter);

uint16_t f32_to_bf16(float f);

}  // namespace wire
}  // namespace dtfs

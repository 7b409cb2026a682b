// Request arena: the host side of zero-copy ingest (serving/arena.py,
// csrc/kernels/ingest.hip share this layout).
//
//   [0]   int32 n_req      [8] int64 total_rows      [16] int64 row_table_off
//   [64]  n_req x {ids_off, wts_off, rows, dst_row} int64 (offsets into payload)
//   [kArenaPayloadOff] payload: serialized PredictRequests (+ scratch for
//                      host-decoded typed fields), then at row_table_off a
//                      {ids_off, wts_off} int32 pair per candidate row
//
// The host parses only protobuf framing and writes descriptors; raw
// tensor_content payloads are referenced in place and the GPU gathers the
// candidate rows. Reference counterpart: the per-shard request construction
// (reference DCNClient.java:91-115), which serialises the same tensors.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace dtfs {
namespace runtime {

constexpr int64_t kArenaPayloadOff = 64 + 32 * 1024;
constexpr int64_t kArenaMaxRequests = 1024;

struct ArenaBatch {
  std::vector<int64_t> rows, offsets;  // per request: candidate rows, first batch row
  std::vector<std::string> errors;     // per request: "" or the INVALID_ARGUMENT message
  int64_t total_rows = 0, used_bytes = 0, n_valid = 0, n_decoded = 0;
};

using Span = std::pair<int64_t, int64_t>;  // (payload offset, length)

// Copy requests into the payload (parallel memcpy); returns their spans.
std::vector<Span> arena_place(uint8_t* arena, int64_t capacity, const std::vector<std::pair<const char*, size_t>>& reqs,
                              int64_t start);

// Parse the requests at `spans` and write header + descriptors. Typed
// (non-tensor_content) fields are decoded into scratch after the last request
// (in parallel over the host pool). Throws std::invalid_argument for spans
// outside the arena or too many requests.
ArenaBatch arena_build(uint8_t* arena, int64_t capacity, const std::vector<Span>& spans, const std::string& ids_key,
                       const std::string& wts_key, int64_t fields, int64_t max_rows);

// Host reference of the GPU unpack: arena -> packed rows [B, W] int64.
void arena_unpack_cpu(const uint8_t* arena, uint8_t* packed, int64_t B, int64_t W, int64_t fields);

}  // namespace runtime
}  // namespace dtfs

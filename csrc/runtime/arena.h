// Request arena: the host side of zero-copy ingest (serving/arena.py,
// csrc/kernels/ingest.hip share this layout).
//
//   [0]   int32 n_req      [8] int64 total_rows      [16] int64 row_table_off
//   [24]  int64 varint_table_off   [32] int32 n_varint_chunks
//   [36]  int32 narrow_wcols (0: narrowed rows carry all F weights)
//   [40]  int32 narrow_id_bytes (3: narrowed rows are packed 3-byte rows; else 4)
//   [64]  n_req x {ids_off, wts_off, rows, dst_row} int64 (offsets into payload)
//   [kArenaPayloadOff] payload: serialized PredictRequests (+ scratch for
//                      host-decoded typed fields), then at row_table_off a
//                      {ids_off, wts_off} int32 pair per candidate row
//
// The host parses only protobuf framing and writes descriptors; raw
// tensor_content payloads (and packed float_val, which is the same bytes) are
// referenced in place and the GPU gathers the candidate rows. Packed varint
// int64_val ids (the reference client's encoding, DCNClient.java:97-108) are
// decoded ON THE GPU when the build allows it (varint_chunks > 0): the host
// cuts each request's varint bytes into kVarintChunk-byte chunks, records per
// chunk the index of its first complete varint (it counts terminator bytes
// anyway to validate the value count), and the varint kernel
// (csrc/kernels/ingest.hip) writes int64 ids into a device-only region after
// the copied bytes, where the row table points. The H2D copy then carries the
// compact wire bytes (~2.4x fewer than tensor_content for the reference's
// requests) instead of host-decoded int64 ids. Reference counterpart: the per-shard request construction
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
constexpr int64_t kVarintChunk = 4096;

// One GPU varint-decode work item (32 bytes; payload-relative offsets).
struct VarintChunk {
  int64_t src_off;    // first byte of this chunk
  int64_t dst_off;    // int64 output array of the request (index 0 = its first id)
  int32_t len;        // bytes in this chunk
  int32_t first_idx;  // index of the first varint that ENDS in this chunk
  int32_t n_values;   // values of the request (bounds)
  int32_t blob_lo;    // bytes of the request's varint run before this chunk (look-back bound)
};
static_assert(sizeof(VarintChunk) == 32, "VarintChunk is shared with the GPU kernel");

struct ArenaBatch {
  std::vector<int64_t> rows, offsets;  // per request: candidate rows, first batch row
  std::vector<std::string> errors;     // per request: "" or the INVALID_ARGUMENT message
  int64_t total_rows = 0, used_bytes = 0, n_valid = 0, n_decoded = 0, n_gpu_varint = 0;
};

using Span = std::pair<int64_t, int64_t>;  // (payload offset, length)

// One request of a batch: a serialized PredictRequest span (parsed here), or
// a request whose candidate features the submitting thread already narrowed
// into the payload (runtime/narrow.h: int32 / 3-byte table rows at ids_off,
// weights of kind wkind - fp32, bf16 or none - at wts_off; payload-relative). A narrow request's row-table entries
// carry bit 31 of ids_off (the GPU reads 4 + 2 bytes per feature there) and
// its descriptor's ids_off carries kNarrowFlag.
struct ArenaItem {
  int64_t off = 0, len = 0;
  bool narrow = false;
  int64_t rows = 0, ids_off = 0, wts_off = 0;
  int wkind = 0;  // narrow: how the weights travel (runtime/narrow.h WtsKind)
};
constexpr int64_t kNarrowFlag = int64_t(1) << 62;

// Copy requests into the payload (parallel memcpy); returns their spans.
std::vector<Span> arena_place(uint8_t* arena, int64_t capacity, const std::vector<std::pair<const char*, size_t>>& reqs,
                              int64_t start);

// Parse the requests at `spans` and write header + descriptors. Typed
// (non-tensor_content) fields are decoded into scratch after the last request
// (in parallel over the host pool). Throws std::invalid_argument for spans
// outside the arena or too many requests.
// varint_chunks: capacity of the GPU varint chunk table (0: packed int64_val
// ids are decoded on the host pool instead).
ArenaBatch arena_build(uint8_t* arena, int64_t capacity, const std::vector<Span>& spans, const std::string& ids_key,
                       const std::string& wts_key, int64_t fields, int64_t max_rows, int64_t varint_chunks = 0);
// Same over a mix of serialized and narrowed requests (results in item order).
// narrow_id_bytes 3: narrowed ids are 3-byte rows (stride 3 F, header @40).
// narrow_wcols > 0: narrowed requests carry only their rows' first
// narrow_wcols weights (row stride 4 * narrow_wcols; header @36 records it, and
// readers see weight 0 for the other columns).
ArenaBatch arena_build_items(uint8_t* arena, int64_t capacity, const std::vector<ArenaItem>& items,
                             const std::string& ids_key, const std::string& wts_key, int64_t fields, int64_t max_rows,
                             int64_t varint_chunks = 0, int64_t narrow_wcols = 0, int64_t narrow_id_bytes = 4);

// Host reference of the GPU varint kernel: fills the arena's device-only id
// region from its chunk table (a no-op when the build decoded on the host).
void arena_varint_cpu(uint8_t* arena);

// Chunk-table capacity that always suffices for `max_rows` x `fields` ids in
// up to `max_requests` requests.
int64_t arena_varint_capacity(int64_t max_rows, int64_t fields, int64_t max_requests);

// Host reference of the GPU unpack: arena -> packed rows [B, W] int64.
void arena_unpack_cpu(const uint8_t* arena, uint8_t* packed, int64_t B, int64_t W, int64_t fields);

}  // namespace runtime
}  // namespace dtfs

// Host-side K0 (input_pack): narrow one request's raw
// candidate ids while they are copied into the pinned arena.
//
//   ids  int64 (tensor_content, any id)  ->  int32 table rows, id mod V
//                                           (python-style non-negative modulo,
//                                           the same rows the GPU hash gives)
//   wts  fp32                           ->  copied as they are, or - when every
//                                           weight of the request is exactly a
//                                           bf16 value - as bf16 (2 bytes), or -
//                                           when every weight is 1.0, the
//                                           reference client's requests
//                                           (DCNClient.java:67-73) - not at all
//
// 8 (7 with 3-byte rows, tables of <= 2^24 rows) instead of 12 bytes per feature cross PCIe, and the narrowing costs about
// what the plain memcpy of the raw bytes it replaces costs (AVX2: the modulo
// runs in double precision with an exact integer correction for ids < 2^52).
// Weights are NOT rounded: a request's scores must not depend on its wire
// encoding (raw tensor_content vs typed fields take different paths); the
// bf16 / implicit forms are chosen only when they are exact.
// Reference counterpart: the client-side tensor building of
// DCNClient.java:97-108, which ships int64 ids and fp32 weights.
#pragma once

#include <cstddef>
#include <cstdint>

namespace dtfs {
namespace runtime {

// How a narrowed request's weights travel (the row table's wts_off bits
// 31..30, csrc/kernels/common.h kWtsOffMask).
enum WtsKind : int { kWtsF32 = 0, kWtsBf16 = 1, kWtsOnes = 2 };
constexpr int64_t kWtsKindShift = 30;
inline int64_t wts_bytes_per(int kind) { return kind == kWtsF32 ? 4 : kind == kWtsBf16 ? 2 : 0; }

// The cheapest exact form of the first wcols fp32 weights of each of `rows`
// rows of `fields` weights (src may be unaligned).
int classify_weights(const uint8_t* src, int64_t rows, int64_t fields, int64_t wcols);
// Those weights stored in `kind` form, wcols per row (kWtsOnes: nothing).
void store_weights(const uint8_t* src, int64_t rows, int64_t fields, int64_t wcols, int kind, uint8_t* dst);

// dst[i] = int32(python_mod(src[i], modulo)); src may be unaligned. modulo in [1, 2^31).
void narrow_ids(const uint8_t* src, int32_t* dst, int64_t n, int64_t modulo);

// The same rows packed into 3 little-endian bytes each (modulo <= 2^24: a
// 1M-row table's rows need 20 bits): dst holds 3 n bytes and may be written up
// to 16 bytes past them (kNarrow24Slack).
constexpr int64_t kNarrow24Slack = 16;
void narrow_ids24(const uint8_t* src, uint8_t* dst, int64_t n, int64_t modulo);

}  // namespace runtime
}  // namespace dtfs

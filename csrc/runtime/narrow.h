// Host-side K0 (input_pack): narrow one request's raw
// candidate features while they are copied into the pinned arena.
//
//   ids  int64 (tensor_content, any id)  ->  int32 table rows, id mod V
//                                           (python-style non-negative modulo,
//                                           the same rows the GPU hash gives)
//   wts  fp32                           ->  bf16 (round to nearest even, NaN kept)
//
// 6 instead of 12 bytes per feature cross PCIe (the DeepFM step's H2D is its
// roofline, profiles/h2d_pacing.md), and the narrowing costs about what the
// plain memcpy of the raw bytes it replaces costs (AVX2: the modulo runs in
// double precision with an exact integer correction for ids < 2^52).
// Reference counterpart: the client-side tensor building of
// DCNClient.java:97-108, which ships int64 ids and fp32 weights.
#pragma once

#include <cstddef>
#include <cstdint>

namespace dtfs {
namespace runtime {

// dst[i] = int32(python_mod(src[i], modulo)); src may be unaligned. modulo in [1, 2^31).
void narrow_ids(const uint8_t* src, int32_t* dst, int64_t n, int64_t modulo);
// dst[i] = bf16(src[i]) (round to nearest even; NaN stays NaN); src may be unaligned.
void narrow_wts(const uint8_t* src, uint16_t* dst, int64_t n);

}  // namespace runtime
}  // namespace dtfs

// K0 (ingest): request bytes -> packed candidate rows, ON THE GPU.
//
// The host only parses protobuf framing: it writes a descriptor per request
// and a {ids_off, wts_off} entry per candidate row into the request arena, and
// DMAs the whole arena - header + raw request bytes + row table - to the device
// with one SDMA copy. This kernel then gathers every candidate row into the
// packed [ids int64 x F | wts fp32 x F | pad] layout the forward reads
// (serving/packing.py). Host memory traffic drops to the DMA read alone, which
// is what lets 8 ranks on one node keep their GPUs fed.
//
// Arena layout: csrc/runtime/arena.h. Offsets inside the payload are arbitrary
// (protobuf does not align tensor_content), so sources are read with aligned
// dword loads + byte funnel shifts and written as aligned 8-byte words.
// Models whose only consumer of ids / weights is the embedding gather skip
// this kernel: the gather reads the arena rows itself (embedding.hip).
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

__global__ void __launch_bounds__(256) unpack_arena_kernel(const uint8_t* __restrict__ arena,
                                                           int64_t* __restrict__ packed, int B, int F, int W) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= B) return;
  const ArenaRow src = arena_row(arena, kArenaPayloadOff, r);
  int64_t* dst = packed + int64_t(r) * W;
  const int ids_bytes = 8 * F, row_bytes = 12 * F;
  // The ids and wts spans are multiples of 4 bytes long, so an output word
  // never straddles them except at the ids|wts boundary, which is 8-aligned in
  // the output (8F bytes).
  for (int c = lane; c < W; c += 64) {
    const int b0 = 8 * c;
    uint64_t v = 0;
    if (src.ids && b0 < row_bytes) {
      if (b0 < ids_bytes) v = load_u64_unaligned(src.ids + b0);
      else if (row_bytes - b0 >= 8) v = load_u64_unaligned(src.wts + (b0 - ids_bytes));
      else v = load_u32_unaligned(src.wts + (b0 - ids_bytes));  // 4-byte wts tail
    }
    dst[c] = int64_t(v);
  }
}

}  // namespace kern

hipError_t launch_unpack_arena(const void* arena, int64_t* packed, int B, int F, int W, int max_req,
                               hipStream_t st) {
  (void)max_req;  // rows are located through the row table, not the descriptors
  if (B == 0) return hipSuccess;
  if (W * 8 < 12 * F) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern::unpack_arena_kernel, dim3((B + 3) / 4), dim3(256), 0, st,
                     static_cast<const uint8_t*>(arena), packed, B, F, W);
  return hipGetLastError();
}

}  // namespace dtfs

// K0 (ingest): request bytes -> packed candidate rows, ON THE GPU.
//
// The host only parses protobuf framing: it writes a descriptor per request
// (where its feat_ids / feat_wts tensor_content payloads sit inside the
// request arena, how many rows it has, which batch row it starts at) and DMAs
// the whole arena - descriptors + raw request bytes - to the device with one
// SDMA copy. This kernel then gathers every candidate row into the packed
// [ids int64 x F | wts fp32 x F | pad] layout the forward reads
// (serving/packing.py). Host memory traffic drops to the DMA read alone, which
// is what lets 8 ranks on one node keep their GPUs fed.
//
// Arena layout (serving/arena.py): header (n_req int32 @0, total_rows int64 @8),
// descriptors at 64: {ids_off, wts_off, rows, dst_row} int64 each, payload at
// kArenaPayloadOff. Offsets inside the payload are arbitrary (protobuf does not
// align tensor_content), so sources are read bytewise and written as aligned
// 8-byte words.
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

__global__ void __launch_bounds__(256) unpack_arena_kernel(const uint8_t* __restrict__ arena,
                                                           int64_t* __restrict__ packed, int B, int F, int W,
                                                           int max_req) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= B) return;
  const int n = min(*reinterpret_cast<const int32_t*>(arena), max_req);
  const int64_t total = *reinterpret_cast<const int64_t*>(arena + 8);
  const int64_t* desc = reinterpret_cast<const int64_t*>(arena + 64);
  const uint8_t* payload = arena + kArenaPayloadOff;
  int64_t* dst = packed + int64_t(r) * W;
  const int ids_bytes = 8 * F, row_bytes = 12 * F;
  const uint8_t* ids_src = nullptr;
  const uint8_t* wts_src = nullptr;
  if (r < total && n > 0) {
    // binary search: last request whose dst_row <= r
    int lo = 0, hi = n - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (desc[4 * mid + 3] <= r) lo = mid;
      else hi = mid - 1;
    }
    const int64_t lr = r - desc[4 * lo + 3];
    if (lr >= 0 && lr < desc[4 * lo + 2]) {
      ids_src = payload + desc[4 * lo + 0] + lr * ids_bytes;
      wts_src = payload + desc[4 * lo + 1] + lr * (4 * F);
    }
  }
  for (int c = lane; c < W; c += 64) {
    const int b0 = 8 * c;
    uint64_t v = 0;
    if (ids_src) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int b = b0 + j;
        uint64_t byte = 0;
        if (b < ids_bytes) byte = ids_src[b];
        else if (b < row_bytes) byte = wts_src[b - ids_bytes];
        v |= byte << (8 * j);
      }
    }
    dst[c] = int64_t(v);
  }
}

}  // namespace kern

hipError_t launch_unpack_arena(const void* arena, int64_t* packed, int B, int F, int W, int max_req,
                               hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (W * 8 < 12 * F) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern::unpack_arena_kernel, dim3((B + 3) / 4), dim3(256), 0, st,
                     static_cast<const uint8_t*>(arena), packed, B, F, W, max_req);
  return hipGetLastError();
}

}  // namespace dtfs

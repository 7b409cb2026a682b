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
  // Each lane produces one aligned 8-byte output word from a possibly
  // misaligned source: three aligned dword loads + byte funnel shifts
  // (v_alignbyte) instead of eight byte loads. The ids and wts spans are
  // multiples of 4 bytes long, so a word never straddles them except at the
  // ids|wts boundary, which is 8-aligned in the output (8F bytes).
  for (int c = lane; c < W; c += 64) {
    const int b0 = 8 * c;
    uint64_t v = 0;
    if (ids_src && b0 < row_bytes) {
      const uint8_t* s = b0 < ids_bytes ? ids_src + b0 : wts_src + (b0 - ids_bytes);
      const int avail = b0 < ids_bytes ? 8 : min(8, row_bytes - b0);  // 8, or 4 at the wts tail
      const uintptr_t a = reinterpret_cast<uintptr_t>(s);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
      const int sh = int(a & 3);
      // load exactly the dwords the span covers (never read past it)
      const uint32_t w0 = w[0];
      const uint32_t w1 = (avail == 8 || sh) ? w[1] : 0u;
      const uint32_t w2 = (avail == 8 && sh) ? w[2] : 0u;
      const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
      const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
      v = avail == 8 ? (uint64_t(hi) << 32) | lo : uint64_t(lo);
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

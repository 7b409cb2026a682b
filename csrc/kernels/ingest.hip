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
#include <algorithm>

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
  if (src.narrow) {  // host-narrowed row: int32 rows -> int64, fp32 weights (packed as 2 per word)
    for (int c = lane; c < W; c += 64) {
      uint64_t v = 0;
      if (c < F) {
        v = uint64_t(arena_narrow_id(src, c));
      } else {
        const int f0 = 2 * (c - F);
        const uint32_t lo = f0 < F ? __float_as_uint(arena_narrow_w(src, f0)) : 0u;
        const uint32_t hi = f0 + 1 < F ? __float_as_uint(arena_narrow_w(src, f0 + 1)) : 0u;
        v = (uint64_t(hi) << 32) | lo;
      }
      dst[c] = int64_t(v);
    }
    return;
  }
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

// Narrow output (the candidate fan-out's exchange rows, serving/packing.py
// PackedLayout(narrow_modulo=m)): [int32 table rows x F | fp32 weights x F],
// 8 bytes per field instead of 12, so the all-to-all moves 2/3 of the bytes.
// Raw ids are hashed (id mod m) here; host-narrowed rows already are.
__global__ void __launch_bounds__(256) unpack_arena_narrow_kernel(const uint8_t* __restrict__ arena,
                                                                  int64_t* __restrict__ packed, int B, int F, int W,
                                                                  int64_t modulo) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= B) return;
  const ArenaRow src = arena_row(arena, kArenaPayloadOff, r);
  int32_t* ids = reinterpret_cast<int32_t*>(packed + int64_t(r) * W);
  float* wts = reinterpret_cast<float*>(ids + F);
  for (int f = lane; f < F; f += 64) {
    int64_t id = 0;
    float w = 0.f;  // padding rows (no request): row 0, weight 0
    if (src.ids) arena_feature(src, f, id, w);
    ids[f] = int32_t(src.narrow ? id : hash_row(id, modulo));
    wts[f] = w;
  }
  // zero the row's pad bytes (fixed-size rows travel whole)
  const int used = 8 * F, total = 8 * W;
  uint8_t* row = reinterpret_cast<uint8_t*>(ids);
  for (int c = used + lane; c < total; c += 64) row[c] = 0;
}

// H2D by the GPU itself: waves read the pinned request arena over PCIe and
// write device memory. Replaces the SDMA copy of the serving step: an SDMA
// command costs 10-17 us of idle engine time between back-to-back copies
// (bench/copy_pipe.py), which on an H2D-paced step is lost throughput. The
// waves are almost all waiting on PCIe reads, use no LDS and few VGPRs, so
// they co-reside with the forward's kernels. U independent 16-B loads per
// lane are in flight (the host side is uncached, coherent memory).
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

template <int U>
__global__ void __launch_bounds__(256) pull_host_kernel(const u32x4_t* __restrict__ src, u32x4_t* __restrict__ dst,
                                                        int64_t n16) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x * U;
  for (int64_t base = int64_t(blockIdx.x) * blockDim.x * U + threadIdx.x; base < n16; base += stride) {
    u32x4_t v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int64_t i = base + int64_t(j) * blockDim.x;
      if (i < n16) v[j] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int64_t i = base + int64_t(j) * blockDim.x;
      if (i < n16) dst[i] = v[j];
    }
  }
}

__global__ void pull_host_tail_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int n) {
  if (int(threadIdx.x) < n) dst[threadIdx.x] = src[threadIdx.x];
}

// Packed varint int64_val ids -> int64, on the GPU (csrc/runtime/arena.h,
// "VarintChunk"). One block per 4096-byte chunk of a request's varint run,
// 16 bytes per lane: a lane finds the terminator bytes (MSB clear) in its
// bytes, a block scan of their counts plus the chunk's first index (from the
// host, which counted terminators to validate the value count) gives each
// varint's index, and the lane holding a terminator decodes that varint by
// walking back over its continuation bytes (<= 9, possibly in the previous
// lane's or chunk's bytes). Blocks loop over chunks (grid is fixed at graph
// capture; the chunk count is read from the arena header).
struct VarintChunkDev {
  int64_t src_off, dst_off;
  int32_t len, first_idx, n_values, blob_lo;
};

__global__ void __launch_bounds__(256) arena_varint_kernel(uint8_t* __restrict__ arena) {
  // chunk bytes staged in LDS behind a 16-byte prefix (a varint is at most 10
  // bytes, so a lane's first varint starts within the previous 16 bytes)
  __shared__ __attribute__((aligned(16))) uint32_t buf[(16 + 4096) / 4];
  __shared__ int wave_tot[4];
  const int n_chunks = *reinterpret_cast<const int32_t*>(arena + 32);
  uint8_t* payload = arena + kArenaPayloadOff;
  const VarintChunkDev* tab =
      reinterpret_cast<const VarintChunkDev*>(payload + *reinterpret_cast<const int64_t*>(arena + 24));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const VarintChunkDev ch = tab[c];
    const uint8_t* src = payload + ch.src_off;
    int64_t* dst = reinterpret_cast<int64_t*>(payload + ch.dst_off);
    const int len = min(ch.len, 4096);
    // stage [src - 16, src + 4096) with aligned dword loads + funnel shifts;
    // bytes before the run read as terminators, past the chunk as continuations
    for (int d = threadIdx.x; d < (16 + 4096) / 4; d += 256) {
      const int k0 = 4 * d - 16;
      uint32_t v = load_u32_unaligned(src + k0);
      if (k0 < -ch.blob_lo || k0 + 4 > len) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + j;
          const uint32_t fill = k < -ch.blob_lo ? 0u : (k >= len ? 0x80u : ((v >> (8 * j)) & 0xffu));
          v = (v & ~(0xffu << (8 * j))) | (fill << (8 * j));
        }
      }
      buf[d] = v;
    }
    __syncthreads();
    const int lo = threadIdx.x * 16;
    const uint4 pw = *reinterpret_cast<const uint4*>(buf + lo / 4);      // the 16 bytes before mine
    const uint4 mw = *reinterpret_cast<const uint4*>(buf + lo / 4 + 4);  // my 16 bytes
    const uint32_t pv[4] = {pw.x, pw.y, pw.z, pw.w}, mv[4] = {mw.x, mw.y, mw.z, mw.w};
    unsigned term = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) term |= unsigned(((mv[j >> 2] >> (8 * (j & 3) + 7)) & 1u) == 0) << j;
    // block exclusive scan of the terminator counts
    const int cnt = __popc(term);
    int incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) wave_tot[wid] = incl;
    __syncthreads();
    int idx = ch.first_idx + incl - cnt;
    for (int q = 0; q < wid; ++q) idx += wave_tot[q];
    // forward scan in registers: the partial varint entering my bytes comes
    // from the previous 16, then every terminator emits one value
    uint64_t acc = 0;
    int sh = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t x = (pv[j >> 2] >> (8 * (j & 3))) & 0xffu;
      if (x & 0x80u) {
        if (sh < 64) acc |= uint64_t(x & 0x7fu) << sh;
        sh += 7;
      } else {
        acc = 0;
        sh = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t x = (mv[j >> 2] >> (8 * (j & 3))) & 0xffu;
      if (sh < 64) acc |= uint64_t(x & 0x7fu) << sh;
      sh += 7;
      if (!(x & 0x80u)) {
        if (idx < ch.n_values) dst[idx] = int64_t(acc);
        ++idx;
        acc = 0;
        sh = 0;
      }
    }
    __syncthreads();  // buf / wave_tot are rewritten by the next chunk
  }
}

}  // namespace kern

const void* arena_varint_kernel_fn() { return reinterpret_cast<const void*>(&kern::arena_varint_kernel); }

hipError_t launch_arena_varint(void* arena, int blocks, hipStream_t st) {
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(kern::arena_varint_kernel, dim3(blocks), dim3(256), 0, st, static_cast<uint8_t*>(arena));
  return hipGetLastError();
}

hipError_t launch_pull_host(void* dst, const void* src, int64_t nbytes, int blocks, hipStream_t st) {
  if (nbytes <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) return hipErrorInvalidValue;
  const int64_t n16 = nbytes / 16;
  const int tail = int(nbytes - n16 * 16);
  if (blocks <= 0) blocks = 128;
  const int64_t need = (n16 + 256 * 4 - 1) / (256 * 4);
  if (need < blocks) blocks = int(std::max<int64_t>(1, need));
  if (n16 > 0)
    hipLaunchKernelGGL(kern::pull_host_kernel<4>, dim3(blocks), dim3(256), 0, st,
                       static_cast<const kern::u32x4_t*>(src), static_cast<kern::u32x4_t*>(dst), n16);
  if (tail)
    hipLaunchKernelGGL(kern::pull_host_tail_kernel, dim3(1), dim3(64), 0, st,
                       static_cast<const uint8_t*>(src) + n16 * 16, static_cast<uint8_t*>(dst) + n16 * 16, tail);
  return hipGetLastError();
}

hipError_t launch_unpack_arena(const void* arena, int64_t* packed, int B, int F, int W, int max_req,
                               hipStream_t st, int64_t narrow_modulo) {
  (void)max_req;  // rows are located through the row table, not the descriptors
  if (B == 0) return hipSuccess;
  if (narrow_modulo > 0) {
    if (W * 8 < 8 * F || narrow_modulo >= (int64_t(1) << 31)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(kern::unpack_arena_narrow_kernel, dim3((B + 3) / 4), dim3(256), 0, st,
                       static_cast<const uint8_t*>(arena), packed, B, F, W, narrow_modulo);
    return hipGetLastError();
  }
  if (W * 8 < 12 * F) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern::unpack_arena_kernel, dim3((B + 3) / 4), dim3(256), 0, st,
                     static_cast<const uint8_t*>(arena), packed, B, F, W);
  return hipGetLastError();
}

}  // namespace dtfs

// Peer lookup kernels (launchers.h PeerLookupArgs, device helpers in
// peer_lookup.h): K1b multi-hot bags over table-wise shards read one-sidedly
// (xGMI loads from the owner's IPC-mapped store instead of an ids + rows
// all-to-all), and the replica cache's maintenance: the fill (hot rows copied
// from their owners into this rank's cache slots) and the open-addressing
// index build. The one-hot step is dot_interact_gather_kernel with the peer
// lookup on (interaction.hip).
#include "common.h"
#include "launchers.h"
#include "peer_lookup.h"

namespace dtfs {
namespace kern {

// 8 lanes per (candidate b, table t): lane c of the group owns columns
// 8c .. 8c + 7 of the pooled row, accumulated in fp32 over the bag's ids.
template <typename IdT>
__global__ void __launch_bounds__(256) peer_bag_kernel(PeerLookupArgs p, const IdT* __restrict__ ids, int64_t ldi,
                                                       const float* __restrict__ wts, int64_t ldw,
                                                       const uint8_t* __restrict__ arena, int col0, int T, int hot,
                                                       int B, bf16* __restrict__ out) {
  const int64_t q = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 3;
  const int c = threadIdx.x & 7;
  const bool valid = q < int64_t(B) * T;
  const int b = valid ? int(q / T) : 0, t = valid ? int(q % T) : 0;
  const CacheView cv = cache_view(p);
  ArenaRow ar{nullptr, nullptr, false, kArenaAllWeights, 4};
  if (arena && valid) ar = arena_row(arena, kArenaPayloadOff, b);
  const int64_t m = p.trows[t];
  const bool sample = valid && c == 0 && p.sample_every > 0 && peer_sampled(p, b);
  const bool counted = valid && c == 0 && peer_counted(p, b);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < hot; ++j) {  // uniform trip count: the ballots below see every lane
    const int col = col0 + t * hot + j;
    int64_t id = 0;
    float w = 0.f;
    if (valid) {
      if (arena) {
        if (ar.ids) arena_feature(ar, col, id, w);
      } else {
        id = int64_t(ids[int64_t(b) * ldi + col]);
        w = wts[int64_t(b) * ldw + col];
      }
    }
    int64_t v = id % m;
    if (v < 0) v += m;
    int hit = -1;
    const bf16* src = peer_row(p, cv, t, v, hit);
    if (valid) {
      const bf16x8 x = *reinterpret_cast<const bf16x8*>(src + c * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += w * bf2f(x[e]);
    }
    peer_count(p, hit, counted);
    ring_push(p, (int64_t(t) << 40) | v, sample && hit >= 0);
  }
  if (valid) {
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    *reinterpret_cast<bf16x8*>(out + q * 64 + c * 8) = o;
  }
}

// 8 lanes per key: rows[slot] = table row of the key, read where it lives
__global__ void __launch_bounds__(256) peer_cache_fill_kernel(PeerLookupArgs p, int T, const int64_t* __restrict__ keys,
                                                              const int32_t* __restrict__ slots, int64_t n,
                                                              bf16* __restrict__ rows, int64_t cap) {
  const int64_t i = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 3;
  const int c = threadIdx.x & 7;
  if (i >= n) return;
  const int64_t key = keys[i];
  const int64_t t = key >> 40;
  const int64_t s = slots[i];
  if (key < 0 || t >= T || s < 0 || s >= cap) return;
  const int64_t v = min(key & ((int64_t(1) << 40) - 1), p.trows[t] - 1);
  const bf16* src = store_row(p, int(t), v);
  *reinterpret_cast<bf16x8*>(rows + s * 64 + c * 8) = *reinterpret_cast<const bf16x8*>(src + c * 8);
}

__global__ void __launch_bounds__(256) cache_index_build_kernel(const int64_t* __restrict__ keys,
                                                                const int32_t* __restrict__ slots, int64_t n,
                                                                int64_t* __restrict__ entries, uint64_t mask) {
  const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t key = keys[i];
  if (key < 0) return;
  uint64_t h = cache_hash(key, mask);
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long*>(entries + 2 * h),
                                             (unsigned long long)kCacheEmpty, (unsigned long long)key);
    if (old == (unsigned long long)kCacheEmpty || old == (unsigned long long)key) {
      entries[2 * h + 1] = slots[i];
      return;
    }
    h = (h + 1) & mask;
  }
}

}  // namespace kern

using namespace kern;

hipError_t launch_peer_bag(const PeerLookupArgs& p, const void* ids, bool ids64, int64_t ldi, const float* wts,
                           int64_t ldw, const void* arena, int col0, int T, int hot, int B, void* out,
                           hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (!p.cbase || !p.towner || !p.toff || !p.trows || !p.tremote || p.max_chunks < 1 || p.chunk_shift < 1 ||
      p.chunk_shift > 40 || T < 1 || hot < 1 || col0 < 0 || !out ||
      (!arena && (!ids || !wts || ldi < col0 + T * hot || ldw < col0 + T * hot)) ||
      (p.ring && (!p.ring_ctr || p.ring_cap < 64)))
    return hipErrorInvalidValue;
  const int64_t threads = int64_t(B) * T * 8;
  const dim3 grid(unsigned((threads + 255) / 256)), block(256);
  const uint8_t* ar = static_cast<const uint8_t*>(arena);
  if (arena || ids64)
    hipLaunchKernelGGL(peer_bag_kernel<int64_t>, grid, block, 0, st, p, static_cast<const int64_t*>(ids), ldi, wts, ldw,
                       ar, col0, T, hot, B, static_cast<bf16*>(out));
  else
    hipLaunchKernelGGL(peer_bag_kernel<int32_t>, grid, block, 0, st, p, static_cast<const int32_t*>(ids), ldi, wts, ldw,
                       ar, col0, T, hot, B, static_cast<bf16*>(out));
  return hipGetLastError();
}

hipError_t launch_peer_cache_fill(const PeerLookupArgs& p, int T, const int64_t* keys, const int32_t* slots,
                                  int64_t n, void* rows, int64_t cap, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!p.cbase || !p.towner || !p.toff || !p.trows || p.max_chunks < 1 || p.chunk_shift < 1 || p.chunk_shift > 40 ||
      !keys || !slots || T < 1 || !rows || cap < 1 || n < 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_cache_fill_kernel, dim3(unsigned((n * 8 + 255) / 256)), dim3(256), 0, st, p, T, keys, slots,
                     n, static_cast<bf16*>(rows), cap);
  return hipGetLastError();
}

hipError_t launch_cache_index_build(const int64_t* keys, const int32_t* slots, int64_t n, int64_t* entries,
                                    int64_t mask, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!keys || !slots || !entries || mask < 1 || ((mask + 1) & mask) || n < 0 || 2 * n > mask + 1)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(cache_index_build_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, keys, slots, n,
                     entries, uint64_t(mask));
  return hipGetLastError();
}

}  // namespace dtfs

// Device side of the peer lookup (launchers.h PeerLookupArgs): a table-wise
// sharded table's row is read where it lives - this rank's store, or the
// owner's store mapped over xGMI by IPC - unless the row is in this rank's
// replica cache of hot remote rows (an open-addressing index over keys
// (t << 40) | row, built by cache_index_build_kernel, immutable while any
// step reads it). Every remote lookup is counted (hit / miss) and rows whose
// candidate index b is a multiple of sample_every push their remote keys into
// a ring the host reads to find the hot rows (parallel/hot_cache.py).
#pragma once
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

constexpr int64_t kCacheEmpty = -1;
constexpr int kCacheMaxProbe = 32;  // the index is built at <= 50 % load
typedef int64_t i64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t cache_hash(int64_t key, uint64_t mask) {
  return ((uint64_t(key) * 0x9E3779B97F4A7C15ull) >> 24) & mask;
}

struct CacheView {
  const int64_t* entries;  // [mask + 1] x {key, slot}: one 16-byte load per probe
  uint64_t mask;           // 0: the cache is empty
  const bf16* rows;
  int64_t cap;
};

__device__ __forceinline__ CacheView cache_view(const PeerLookupArgs& p) {
  CacheView c{nullptr, 0, nullptr, 0};
  if (p.cache) {
    // the host swaps indices by rewriting the single word cache[0]
    c.entries = reinterpret_cast<const int64_t*>(p.cache[0]);
    c.mask = uint64_t(p.cache[2]);
    c.rows = reinterpret_cast<const bf16*>(p.cache[3]);
    c.cap = p.cache[4];
    if (!c.entries || !c.rows || c.cap < 1) c.mask = 0;
  }
  return c;
}

// Row v of table t where it lives (its owner's store chunk)
__device__ __forceinline__ const bf16* store_row(const PeerLookupArgs& p, int t, int64_t v) {
  const int64_t g = p.toff[t] + v;
  const int64_t c = int64_t(p.towner[t]) * p.max_chunks + (g >> p.chunk_shift);
  return reinterpret_cast<const bf16*>(p.cbase[c]) + (g & ((int64_t(1) << p.chunk_shift) - 1)) * 64;
}

__device__ __forceinline__ const bf16* peer_row(const PeerLookupArgs& p, const CacheView& c, int t, int64_t v,
                                                int& hit) {
  const bf16* src = store_row(p, t, v);
  hit = -1;
  if (p.tremote[t]) {
    hit = 0;
    if (c.mask) {
      const int64_t key = (int64_t(t) << 40) | v;
      uint64_t h = cache_hash(key, c.mask);
      for (int probe = 0; probe < kCacheMaxProbe; ++probe) {
        const i64x2 e = *reinterpret_cast<const i64x2*>(c.entries + 2 * h);
        const int64_t k = e[0];
        if (k == key) {
          const int64_t s = e[1];
          if (s >= 0 && s < c.cap) {
            src = c.rows + s * 64;
            hit = 1;
          }
          break;
        }
        if (k == kCacheEmpty) break;
        h = (h + 1) & c.mask;
      }
    }
  }
  return src;
}

// Candidates whose remote keys are sampled for the hot set (b % sample_every
// == 0) and, disjoint from them, candidates whose lookups are counted (b %
// sample_every == sample_every / 2): a repeating request stream then cannot
// report its own samples back as hits. sample_every <= 1: every candidate is
// both. Counting a subset keeps the counters' atomics (one per wave and kind,
// on 128 addresses) off most waves - counting every lookup cost ~3 us per
// 16384-candidate step (tools/studies/peer_lookup_bench.py).
// The sampling period: word 1 of the cache descriptor when > 0 (set by the
// host between steps - HotRowCache.set_sample_period: every candidate while
// the cache learns, the captured graphs unchanged), else sample_every.
__device__ __forceinline__ int64_t peer_sample_period(const PeerLookupArgs& p) {
  const int64_t dyn = p.cache ? p.cache[1] : 0;
  return dyn > 0 ? dyn : int64_t(p.sample_every);
}
__device__ __forceinline__ bool peer_sampled(const PeerLookupArgs& p, int64_t b) {
  const int64_t sp = peer_sample_period(p);
  return sp <= 1 || b % sp == 0;
}
__device__ __forceinline__ bool peer_counted(const PeerLookupArgs& p, int64_t b) {
  return p.sample_every <= 1 || b % p.sample_every == p.sample_every / 2;
}

// Wave-aggregated counters: one atomic per wave and kind. Called by every
// lane of the wave (ballots); lanes with counted = false contribute nothing.
__device__ __forceinline__ void peer_count(const PeerLookupArgs& p, int hit, bool counted) {
  if (!p.stats) return;
  const uint64_t hits = __ballot(counted && hit == 1), miss = __ballot(counted && hit == 0);
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    unsigned long long* s = p.stats + 2 * (blockIdx.x & 63);
    if (hits) atomicAdd(s, (unsigned long long)__popcll(hits));
    if (miss) atomicAdd(s + 1, (unsigned long long)__popcll(miss));
  }
}

// Push the keys of the active lanes into the sample ring: 64 segments of
// ring_cap / 64 keys, each with its own write counter ring_ctr[block % 64]
// (wrapping), so the pushes of concurrent waves spread over 64 addresses.
__device__ __forceinline__ void ring_push(const PeerLookupArgs& p, int64_t key, bool active) {
  if (!p.ring || p.ring_cap < 64) return;
  const uint64_t m = __ballot(active);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  const int seg = blockIdx.x & 63;
  const uint64_t seg_cap = uint64_t(p.ring_cap) / 64;
  unsigned long long base = 0;
  if (lane == leader) base = atomicAdd(p.ring_ctr + seg, (unsigned long long)__popcll(m));
  const uint32_t lo = __shfl(uint32_t(base), leader), hi = __shfl(uint32_t(base >> 32), leader);
  base = (uint64_t(hi) << 32) | lo;
  if (active) {
    const int below = __popcll(m & ((1ull << lane) - 1ull));
    p.ring[int64_t(seg * seg_cap + (base + below) % seg_cap)] = key;
  }
}

}  // namespace kern
}  // namespace dtfs

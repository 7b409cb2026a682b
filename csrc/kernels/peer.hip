// One-shot peer exchange over IPC-mapped mailboxes (SURVEY.md §2.5 C1/C2
// "one-shot direct all-gather over all 7 xGMI links, not a ring"; §7 step 6
// "benchmark a one-shot peer-copy alternative").
//
// The reference's fan-out is one RPC per shard and a join
// (reference DCNClient.java:146-164): every message goes straight to its
// destination. On an MI355X node the same shape is a single kernel per rank:
// block p PUSHES this rank's message for peer p into p's mailbox with plain
// vector stores over xGMI, raises p's flag for this sequence number, then
// waits for p's flag in its own mailbox and copies p's message out. No ring,
// no proxy thread, no protocol selection: one launch and one xGMI hop per
// message, which is what a <= 64 KB latency-bound exchange (the per-step score
// gather, a single request's row scatter) wants.
//
// Mailbox of one rank (uncached device memory, exported with hipIpcGetMemHandle):
//   flag[slot][src]  u64, 64-byte stride    - sequence number of src's message
//   ack[src]         u64, 64-byte stride    - last sequence this rank's message
//                                             to src was consumed by src
//   data[slot][src]  cap bytes              - src's message
// `slot` = seq % kPeerDepth, so kPeerDepth exchanges can be in flight before a
// sender has to wait for its peer's ack (back-pressure instead of a barrier).
// The sequence number lives in device memory (ctl->seq) and is advanced by the
// last block of each exchange, so the launch is graph-capturable and needs no
// host bookkeeping. Every spin is bounded (s_memrealtime, 100 MHz): a peer that
// never answers makes the kernel record an error word in mapped host memory,
// fill the receive buffers it could not deliver with all-ones (NaN scores) and
// exit, so the grid always drains; the host reports it through
// RcclComm::async_error(), which the step wait checks once more before it
// declares a step done, and further exchanges on the communicator throw.
#include "common.h"
#include "peer_exchange.h"

namespace dtfs {
namespace kern {

namespace {

__device__ __forceinline__ uint64_t ld_acquire(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_release(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Copy n bytes with the whole block: 16 B per lane when both ends allow it.
__device__ __forceinline__ void block_copy(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint64_t n) {
  const int t = threadIdx.x, nt = blockDim.x;
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
    const uint64_t n16 = n >> 4;
    const i32x4* s = reinterpret_cast<const i32x4*>(src);
    i32x4* d = reinterpret_cast<i32x4*>(dst);
    for (uint64_t i = t; i < n16; i += nt) d[i] = s[i];
    for (uint64_t i = (n16 << 4) + t; i < n; i += nt) dst[i] = src[i];
  } else if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 3) == 0) {
    const uint64_t n4 = n >> 2;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t i = t; i < n4; i += nt) d[i] = s[i];
    for (uint64_t i = (n4 << 2) + t; i < n; i += nt) dst[i] = src[i];
  } else {
    for (uint64_t i = t; i < n; i += nt) dst[i] = src[i];
  }
}

// Thread 0 spins until *p satisfies the predicate or the deadline passes.
// Returns false on timeout. Wave-uniform exit: only lane 0 of wave 0 calls it.
template <typename Pred>
__device__ bool spin_until(const uint64_t* p, Pred ok, uint64_t deadline) {
  for (;;) {
    if (ok(ld_acquire(p))) return true;
    if (__builtin_amdgcn_s_memrealtime() > deadline) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

__global__ void __launch_bounds__(256) peer_exchange_kernel(PeerExchangeArgs a) {
  const int p = blockIdx.x;  // the peer this block serves
  const int me = a.rank;
  __shared__ uint64_t s_seq;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    s_seq = a.ctl->seq + 1;
    s_ok = a.ctl->broken == 0;
  }
  __syncthreads();
  const uint64_t seq = s_seq;
  const int slot = int(seq % kPeerDepth);
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + a.timeout_ticks;

  if (s_ok) {
    if (p == me) {
      block_copy(a.dst[p], a.src[p], a.send_bytes[p]);
    } else {
      uint8_t* rbox = a.box[p];   // peer p's mailbox (IPC-mapped)
      uint8_t* lbox = a.box[me];  // this rank's mailbox
      // 1. back-pressure: p has consumed this rank's message of seq - depth
      if (threadIdx.x == 0) {
        const uint64_t need = seq > kPeerDepth ? seq - kPeerDepth : 0;
        if (!spin_until(peer_ack(lbox, p), [need](uint64_t v) { return v >= need; }, deadline)) s_ok = 0;
      }
      __syncthreads();
      if (s_ok) {
        // 2. push: data into p's slot for this rank, then the flag (release)
        if (a.send_bytes[p]) block_copy(peer_data(rbox, slot, me, a.cap, a.nranks), a.src[p], a.send_bytes[p]);
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) {
          st_release(peer_flag(rbox, slot, me), seq);
          // 3. receive: p's flag for this sequence in this rank's mailbox
          if (!spin_until(peer_flag(lbox, slot, p), [seq](uint64_t v) { return v == seq; }, deadline)) s_ok = 0;
        }
        __syncthreads();
        if (s_ok) {
          if (a.recv_bytes[p]) block_copy(a.dst[p], peer_data(lbox, slot, p, a.cap, a.nranks), a.recv_bytes[p]);
          __syncthreads();  // every lane's read of the slot is done
          if (threadIdx.x == 0) st_release(peer_ack(rbox, me), seq);  // 4. slot free again
        }
      }
    }
  }
  __syncthreads();
  if (!s_ok && a.dst[p] && a.recv_bytes[p]) {
    // poison what this block should have delivered (all-ones: NaN as fp32
    // scores, -1 as int32 rows - which the gather clamps): a host that misses
    // the error word cannot hand out plausible-looking scores from stale data
    uint8_t* d = a.dst[p];
    const uint64_t n = a.recv_bytes[p];
    if ((reinterpret_cast<uintptr_t>(d) & 3) == 0) {
      for (uint64_t i = threadIdx.x; i < (n >> 2); i += blockDim.x) reinterpret_cast<uint32_t*>(d)[i] = 0xffffffffu;
      for (uint64_t i = ((n >> 2) << 2) + threadIdx.x; i < n; i += blockDim.x) d[i] = 0xff;
    } else {
      for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = 0xff;
    }
  }
  if (threadIdx.x == 0) {
    if (!s_ok) {
      a.ctl->broken = 1;
      *a.err_host = 1;  // mapped host word: the host's async_error() sees it
      __threadfence_system();
    }
    // last block out advances the sequence (every block has read it by now)
    const unsigned prev = atomicAdd(&a.ctl->done, 1u);
    if (prev == gridDim.x - 1) {
      a.ctl->done = 0;
      a.ctl->seq = seq;
      __threadfence();
    }
  }
}

}  // namespace
}  // namespace kern

hipError_t launch_peer_exchange(const PeerExchangeArgs& a, hipStream_t st) {
  if (a.nranks < 1 || a.nranks > kPeerMaxRanks || a.rank < 0 || a.rank >= a.nranks) return hipErrorInvalidValue;
  for (int p = 0; p < a.nranks; ++p)
    if (a.send_bytes[p] > a.cap || a.recv_bytes[p] > a.cap) return hipErrorInvalidValue;
  hipLaunchKernelGGL(kern::peer_exchange_kernel, dim3(a.nranks), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace dtfs

// Layout and launch interface of the one-shot peer exchange (peer.hip), shared
// by the kernel and the host side that allocates / maps the mailboxes
// (csrc/comm/rccl_comm.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtfs {

constexpr int kPeerMaxRanks = 16;  // one node: 8 GPUs (16 = one-GPU rehearsals with extra ranks)
constexpr int kPeerDepth = 4;      // exchanges in flight before a sender waits for its peer's ack
constexpr int kPeerLine = 64;      // flag / ack stride (one per cache line)

// Per-rank control block in ordinary device memory (never shared).
struct PeerCtl {
  uint64_t seq;     // sequence number of the last completed exchange
  unsigned done;    // blocks of the running exchange that finished
  unsigned broken;  // a spin timed out: every later exchange is skipped
};

constexpr uint64_t kPeerHeaderBytes = uint64_t(kPeerDepth + 1) * kPeerMaxRanks * kPeerLine;
__host__ __device__ inline uint64_t peer_box_bytes(int nranks, uint64_t cap) {
  return kPeerHeaderBytes + uint64_t(kPeerDepth) * nranks * cap;
}
__host__ __device__ inline uint64_t* peer_flag(uint8_t* box, int slot, int src) {
  return reinterpret_cast<uint64_t*>(box + (uint64_t(slot) * kPeerMaxRanks + src) * kPeerLine);
}
__host__ __device__ inline uint64_t* peer_ack(uint8_t* box, int src) {
  return reinterpret_cast<uint64_t*>(box + (uint64_t(kPeerDepth) * kPeerMaxRanks + src) * kPeerLine);
}
__host__ __device__ inline uint8_t* peer_data(uint8_t* box, int slot, int src, uint64_t cap, int nranks) {
  return box + kPeerHeaderBytes + (uint64_t(slot) * nranks + src) * cap;
}

struct PeerExchangeArgs {
  int rank = 0, nranks = 1;
  uint64_t cap = 0;                  // bytes per (slot, source) message
  uint64_t timeout_ticks = 0;        // s_memrealtime ticks (100 MHz) per spin
  uint8_t* box[kPeerMaxRanks] = {};  // every rank's mailbox, mapped into this process (own one local)
  const uint8_t* src[kPeerMaxRanks] = {};  // this rank's message for peer p
  uint8_t* dst[kPeerMaxRanks] = {};        // where peer p's message to this rank lands
  uint64_t send_bytes[kPeerMaxRanks] = {};
  uint64_t recv_bytes[kPeerMaxRanks] = {};
  PeerCtl* ctl = nullptr;
  int* err_host = nullptr;  // mapped pinned host word (device pointer)
};

hipError_t launch_peer_exchange(const PeerExchangeArgs& a, hipStream_t st);

}  // namespace dtfs

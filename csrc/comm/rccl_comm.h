// Native RCCL communicator for the candidate fan-out (SURVEY.md §2.3
// "csrc/comm/rccl_fanout.cpp", collectives C1/C2).
//
// The reference fans candidates out over per-host gRPC channels (reference
// DCNClient.java:118-135 channels, :146-164 dispatch/join). Inside one MI355X
// node the hop is xGMI, and the collectives are issued from C++ straight onto
// HIP streams by the StepRunner, so a fan-out step costs no Python and no
// ProcessGroup bookkeeping per step. Bootstrap reuses torch.distributed only
// to broadcast the 128-byte ncclUniqueId.
//
// Every message of a step has a static size (equal per-rank splits), so the
// ops are plain ncclAllToAll / grouped send-recv with no count exchange.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace dtfs {
namespace comm {

// Path of the librccl to use (PyTorch's bundled copy); must be set before the
// first RCCL call. Symbols are resolved with dlopen/dlsym, nothing is linked.
void set_library(const std::string& path);
std::string unique_id();  // ncclGetUniqueId, as raw bytes

class RcclComm {
 public:
  RcclComm(const std::string& uid, int nranks, int rank, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int nranks() const { return nranks_; }

  // recv[r] = rank r's send[me]; `bytes` per peer.
  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t st);
  // root's send[r] -> rank r's recv (bytes each). send is only read on root.
  void scatter(const void* send, void* recv, size_t bytes, int root, hipStream_t st);
  // every rank's send -> root's recv[r] (bytes each).
  void gather(const void* send, void* recv, size_t bytes, int root, hipStream_t st);
  // recv[r] = rank r's send.
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t st);

  // recv = this rank's `elems`-long slice of the element-wise bf16 sum of every
  // rank's send (W x elems). Row-wise sharded embedding tables: exactly one
  // rank contributes a non-zero row, so the bf16 sum is exact.
  void reduce_scatter_bf16(const void* send, void* recv, size_t elems, hipStream_t st);

  // One-shot peer exchange (csrc/kernels/peer.hip): alltoall / scatter /
  // gather / allgather messages of at most `cap` bytes per peer go through
  // IPC-mapped mailboxes in ONE kernel per rank instead of RCCL. Setup is
  // collective: every rank calls peer_prepare (allocates and exports its
  // mailbox), the handles are exchanged out of band (torch.distributed), then
  // every rank calls peer_enable with all handles in rank order.
  // Like the RCCL collectives, one communicator's exchanges must be issued in
  // the same order on every rank and stream-ordered (one stream per
  // communicator): the sequence number advances kernel by kernel.
  std::string peer_prepare(uint64_t cap);
  // hipDeviceCanAccessPeer from this communicator's device (1 for itself)
  bool can_access_device(int peer_device) const;
  void peer_enable(const std::vector<std::string>& handles, double timeout_s);
  bool peer_enabled() const { return peer_ && peer_->enabled; }
  uint64_t peer_cap() const { return peer_ ? peer_->cap : 0; }
  uint64_t peer_exchanges() const { return peer_ ? peer_->count : 0; }

  // "" when healthy, else the asynchronous RCCL error (failure detection).
  std::string async_error();
  // throws if the communicator is aborted or its peer exchange timed out
  void check_usable() const;
  // Abort in-flight operations (a peer died / a deadline passed); the
  // communicator is unusable afterwards.
  void abort();
  bool aborted() const { return aborted_; }

 private:
  void check(ncclResult_t r, const char* what);
  struct Peer {
    uint64_t cap = 0;
    bool enabled = false;
    uint64_t count = 0;
    double timeout_s = 5.0;
    uint8_t* box = nullptr;               // own mailbox
    std::vector<uint8_t*> boxes;          // every rank's, mapped (own one local)
    std::vector<bool> opened;             // which were opened from an IPC handle
    void* ctl = nullptr;                  // PeerCtl, device memory
    int* err_host = nullptr;              // mapped pinned word set by a timed-out kernel
    int* err_dev = nullptr;
  };
  // true when the exchange went through the mailboxes
  bool peer_run(const void* const* src, void* const* dst, const uint64_t* send_bytes, const uint64_t* recv_bytes,
                hipStream_t st);
  void peer_release();
  std::unique_ptr<Peer> peer_;
  ncclComm_t comm_ = nullptr;
  int nranks_ = 1, rank_ = 0, device_ = 0;
  bool aborted_ = false;
};

}  // namespace comm
}  // namespace dtfs

#include "rccl_comm.h"

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <stdexcept>

#include "kernels/peer_exchange.h"

namespace dtfs {
namespace comm {

namespace {

// RCCL entry points, resolved from the librccl that PyTorch already loaded
// (ProcessGroupNCCL's), so the process holds exactly one RCCL instance: one
// set of proxy threads, one IPC/bootstrap state, one version across ranks.
struct Api {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclAllToAll) AllToAll = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclReduceScatter) ReduceScatter = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
};
Api g_api;
std::once_flag g_once;
std::string g_path, g_err;

template <typename F>
void sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  if (!out) throw std::runtime_error(std::string("RCCL symbol missing: ") + name);
}

const Api& api() {
  std::call_once(g_once, [] {
    try {
      if (g_path.empty()) throw std::runtime_error("set_library() was not called");
      void* h = dlopen(g_path.c_str(), RTLD_NOW | RTLD_NOLOAD);  // the instance torch loaded
      if (!h) h = dlopen(g_path.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (!h) throw std::runtime_error(std::string("dlopen ") + g_path + ": " + dlerror());
      sym(h, "ncclGetUniqueId", g_api.GetUniqueId);
      sym(h, "ncclCommInitRank", g_api.CommInitRank);
      sym(h, "ncclCommDestroy", g_api.CommDestroy);
      sym(h, "ncclCommAbort", g_api.CommAbort);
      sym(h, "ncclCommGetAsyncError", g_api.CommGetAsyncError);
      sym(h, "ncclGetErrorString", g_api.GetErrorString);
      sym(h, "ncclAllToAll", g_api.AllToAll);
      sym(h, "ncclAllGather", g_api.AllGather);
      sym(h, "ncclReduceScatter", g_api.ReduceScatter);
      sym(h, "ncclSend", g_api.Send);
      sym(h, "ncclRecv", g_api.Recv);
      sym(h, "ncclGroupStart", g_api.GroupStart);
      sym(h, "ncclGroupEnd", g_api.GroupEnd);
    } catch (const std::exception& e) {
      g_err = e.what();
    }
  });
  if (!g_err.empty()) throw std::runtime_error("RCCL unavailable: " + g_err);
  return g_api;
}

void ck_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

void set_library(const std::string& path) {
  if (g_path.empty()) g_path = path;
}

std::string unique_id() {
  const Api& a = api();
  ncclUniqueId id;
  ncclResult_t r = a.GetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error(std::string("ncclGetUniqueId: ") + a.GetErrorString(r));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

RcclComm::RcclComm(const std::string& uid, int nranks, int rank, int device)
    : nranks_(nranks), rank_(rank), device_(device) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("bad rank / nranks");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  ck_hip(hipSetDevice(device), "hipSetDevice");
  check(api().CommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() {
  peer_release();
  if (!comm_ || aborted_) return;  // an aborted communicator is already released
  hipSetDevice(device_);
  const Api& a = api();
  ncclResult_t async = ncclSuccess;
  a.CommGetAsyncError(comm_, &async);
  if (async != ncclSuccess) a.CommAbort(comm_);
  else a.CommDestroy(comm_);
}

void RcclComm::check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string(what) + ": " + api().GetErrorString(r));
}

void RcclComm::alltoall(const void* send, void* recv, size_t bytes, hipStream_t st) {
  check_usable();
  if (peer_enabled() && bytes <= peer_->cap) {
    const void* src[kPeerMaxRanks];
    void* dst[kPeerMaxRanks];
    uint64_t n[kPeerMaxRanks];
    for (int p = 0; p < nranks_; ++p) {
      src[p] = static_cast<const uint8_t*>(send) + size_t(p) * bytes;
      dst[p] = static_cast<uint8_t*>(recv) + size_t(p) * bytes;
      n[p] = bytes;
    }
    if (peer_run(src, dst, n, n, st)) return;
  }
  check(api().AllToAll(send, recv, bytes, ncclUint8, comm_, st), "ncclAllToAll");
}

void RcclComm::scatter(const void* send, void* recv, size_t bytes, int root, hipStream_t st) {
  check_usable();
  if (peer_enabled() && bytes <= peer_->cap) {
    const void* src[kPeerMaxRanks] = {};
    void* dst[kPeerMaxRanks] = {};
    uint64_t ns[kPeerMaxRanks] = {}, nr[kPeerMaxRanks] = {};
    for (int p = 0; p < nranks_ && rank_ == root; ++p) {
      src[p] = static_cast<const uint8_t*>(send) + size_t(p) * bytes;
      ns[p] = bytes;
    }
    dst[root] = recv;
    nr[root] = bytes;
    if (peer_run(src, dst, ns, nr, st)) return;
  }
  const Api& a = api();
  check(a.GroupStart(), "ncclGroupStart");
  if (rank_ == root) {
    const uint8_t* s = static_cast<const uint8_t*>(send);
    for (int r = 0; r < nranks_; ++r) check(a.Send(s + size_t(r) * bytes, bytes, ncclUint8, r, comm_, st), "ncclSend");
  }
  check(a.Recv(recv, bytes, ncclUint8, root, comm_, st), "ncclRecv");
  check(a.GroupEnd(), "ncclGroupEnd");
}

void RcclComm::gather(const void* send, void* recv, size_t bytes, int root, hipStream_t st) {
  check_usable();
  if (peer_enabled() && bytes <= peer_->cap) {
    const void* src[kPeerMaxRanks] = {};
    void* dst[kPeerMaxRanks] = {};
    uint64_t ns[kPeerMaxRanks] = {}, nr[kPeerMaxRanks] = {};
    src[root] = send;
    ns[root] = bytes;
    for (int p = 0; p < nranks_ && rank_ == root; ++p) {
      dst[p] = static_cast<uint8_t*>(recv) + size_t(p) * bytes;
      nr[p] = bytes;
    }
    if (peer_run(src, dst, ns, nr, st)) return;
  }
  const Api& a = api();
  check(a.GroupStart(), "ncclGroupStart");
  if (rank_ == root) {
    uint8_t* d = static_cast<uint8_t*>(recv);
    for (int r = 0; r < nranks_; ++r) check(a.Recv(d + size_t(r) * bytes, bytes, ncclUint8, r, comm_, st), "ncclRecv");
  }
  check(a.Send(send, bytes, ncclUint8, root, comm_, st), "ncclSend");
  check(a.GroupEnd(), "ncclGroupEnd");
}

void RcclComm::allgather(const void* send, void* recv, size_t bytes, hipStream_t st) {
  check_usable();
  if (peer_enabled() && bytes <= peer_->cap) {
    const void* src[kPeerMaxRanks];
    void* dst[kPeerMaxRanks];
    uint64_t n[kPeerMaxRanks];
    for (int p = 0; p < nranks_; ++p) {
      src[p] = send;
      dst[p] = static_cast<uint8_t*>(recv) + size_t(p) * bytes;
      n[p] = bytes;
    }
    if (peer_run(src, dst, n, n, st)) return;
  }
  check(api().AllGather(send, recv, bytes, ncclUint8, comm_, st), "ncclAllGather");
}

void RcclComm::reduce_scatter_bf16(const void* send, void* recv, size_t elems, hipStream_t st) {
  check_usable();
  check(api().ReduceScatter(send, recv, elems, ncclBfloat16, ncclSum, comm_, st), "ncclReduceScatter");
}

void RcclComm::check_usable() const {
  if (aborted_) throw std::runtime_error("communicator aborted");
  // a timed-out peer exchange is sticky (its sequence numbers no longer match
  // the peers'): launching more would move no data and report success
  if (peer_ && peer_->err_host && __atomic_load_n(peer_->err_host, __ATOMIC_ACQUIRE))
    throw std::runtime_error("communicator broken: a peer exchange timed out (a peer rank stopped answering)");
}

std::string RcclComm::async_error() {
  if (aborted_) return "aborted";
  if (peer_ && peer_->err_host && __atomic_load_n(peer_->err_host, __ATOMIC_ACQUIRE))
    return "peer exchange timed out (a peer rank stopped answering)";
  const Api& a = api();
  ncclResult_t async = ncclSuccess;
  ncclResult_t r = a.CommGetAsyncError(comm_, &async);
  if (r != ncclSuccess) return a.GetErrorString(r);
  if (async != ncclSuccess && async != ncclInProgress) return a.GetErrorString(async);
  return "";
}

void RcclComm::abort() {
  if (aborted_ || !comm_) return;
  hipSetDevice(device_);
  api().CommAbort(comm_);
  aborted_ = true;
}

// ---- one-shot peer exchange --------------------------------------------------

bool RcclComm::can_access_device(int peer_device) const {
  if (peer_device == device_) return true;
  int ok = 0;
  if (hipDeviceCanAccessPeer(&ok, device_, peer_device) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return ok != 0;
}

std::string RcclComm::peer_prepare(uint64_t cap) {
  if (peer_) throw std::runtime_error("peer exchange already prepared");
  if (nranks_ > kPeerMaxRanks) throw std::invalid_argument("peer exchange: too many ranks");
  cap = (std::max<uint64_t>(cap, 256) + 255) & ~uint64_t(255);
  ck_hip(hipSetDevice(device_), "hipSetDevice");
  auto pe = std::make_unique<Peer>();
  pe->cap = cap;
  const uint64_t bytes = peer_box_bytes(nranks_, cap);
  // uncached: peers write it over xGMI while this GPU polls it, and neither
  // side's L2 may hold a stale copy of a flag or a slot
  ck_hip(hipExtMallocWithFlags(reinterpret_cast<void**>(&pe->box), bytes, hipDeviceMallocUncached),
         "hipExtMallocWithFlags(peer mailbox)");
  ck_hip(hipMemset(pe->box, 0, bytes), "hipMemset(peer mailbox)");
  ck_hip(hipMalloc(&pe->ctl, sizeof(PeerCtl)), "hipMalloc(peer ctl)");
  ck_hip(hipMemset(pe->ctl, 0, sizeof(PeerCtl)), "hipMemset(peer ctl)");
  ck_hip(hipHostMalloc(reinterpret_cast<void**>(&pe->err_host), sizeof(int), hipHostMallocMapped),
         "hipHostMalloc(peer err)");
  *pe->err_host = 0;
  ck_hip(hipHostGetDevicePointer(reinterpret_cast<void**>(&pe->err_dev), pe->err_host, 0), "hipHostGetDevicePointer");
  ck_hip(hipDeviceSynchronize(), "hipDeviceSynchronize(peer prepare)");
  hipIpcMemHandle_t h;
  ck_hip(hipIpcGetMemHandle(&h, pe->box), "hipIpcGetMemHandle(peer mailbox)");
  peer_ = std::move(pe);
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void RcclComm::peer_enable(const std::vector<std::string>& handles, double timeout_s) {
  if (!peer_) throw std::runtime_error("peer_prepare() first");
  if (peer_->enabled) return;
  if (int(handles.size()) != nranks_) throw std::invalid_argument("peer_enable: one handle per rank");
  ck_hip(hipSetDevice(device_), "hipSetDevice");
  peer_->timeout_s = timeout_s > 0 ? timeout_s : 5.0;
  peer_->boxes.assign(size_t(nranks_), nullptr);
  peer_->opened.assign(size_t(nranks_), false);
  for (int p = 0; p < nranks_; ++p) {
    if (p == rank_) {
      peer_->boxes[size_t(p)] = peer_->box;
      continue;
    }
    if (handles[size_t(p)].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("peer_enable: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[size_t(p)].data(), sizeof(h));
    void* ptr = nullptr;
    ck_hip(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(peer mailbox)");
    peer_->boxes[size_t(p)] = static_cast<uint8_t*>(ptr);
    peer_->opened[size_t(p)] = true;
  }
  peer_->enabled = true;
}

bool RcclComm::peer_run(const void* const* src, void* const* dst, const uint64_t* send_bytes,
                        const uint64_t* recv_bytes, hipStream_t st) {
  PeerExchangeArgs a;
  a.rank = rank_;
  a.nranks = nranks_;
  a.cap = peer_->cap;
  a.timeout_ticks = uint64_t(peer_->timeout_s * 1e8);  // s_memrealtime: 100 MHz
  for (int p = 0; p < nranks_; ++p) {
    a.box[p] = peer_->boxes[size_t(p)];
    a.src[p] = static_cast<const uint8_t*>(src[p]);
    a.dst[p] = static_cast<uint8_t*>(dst[p]);
    a.send_bytes[p] = src[p] ? send_bytes[p] : 0;
    a.recv_bytes[p] = dst[p] ? recv_bytes[p] : 0;
  }
  a.ctl = static_cast<PeerCtl*>(peer_->ctl);
  a.err_host = peer_->err_dev;
  ck_hip(launch_peer_exchange(a, st), "peer exchange launch");
  ++peer_->count;
  return true;
}

void RcclComm::peer_release() {
  if (!peer_) return;
  hipSetDevice(device_);
  for (size_t p = 0; p < peer_->boxes.size(); ++p)
    if (peer_->opened[p]) hipIpcCloseMemHandle(peer_->boxes[p]);
  if (peer_->box) hipFree(peer_->box);
  if (peer_->ctl) hipFree(peer_->ctl);
  if (peer_->err_host) hipHostFree(peer_->err_host);
  peer_.reset();
}

}  // namespace comm
}  // namespace dtfs

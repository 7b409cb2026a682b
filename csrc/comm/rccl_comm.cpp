#include "rccl_comm.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

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
  if (aborted_) throw std::runtime_error("communicator aborted");
  check(api().AllToAll(send, recv, bytes, ncclUint8, comm_, st), "ncclAllToAll");
}

void RcclComm::scatter(const void* send, void* recv, size_t bytes, int root, hipStream_t st) {
  if (aborted_) throw std::runtime_error("communicator aborted");
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
  if (aborted_) throw std::runtime_error("communicator aborted");
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
  if (aborted_) throw std::runtime_error("communicator aborted");
  check(api().AllGather(send, recv, bytes, ncclUint8, comm_, st), "ncclAllGather");
}

void RcclComm::reduce_scatter_bf16(const void* send, void* recv, size_t elems, hipStream_t st) {
  if (aborted_) throw std::runtime_error("communicator aborted");
  check(api().ReduceScatter(send, recv, elems, ncclBfloat16, ncclSum, comm_, st), "ncclReduceScatter");
}

std::string RcclComm::async_error() {
  if (aborted_) return "aborted";
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

}  // namespace comm
}  // namespace dtfs

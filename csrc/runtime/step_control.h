// Intra-node step agreement for a multi-rank live server (one process per GPU).
//
// Every rank of a candidate fan-out must launch the same steps, in the same
// order, with the same padding bucket: each step's collectives pair up across
// ranks. The round-2 design launched the LARGEST bucket on every rank on a
// fixed cadence (empty steps every batch timeout, forever). Here a step exists
// only when some rank has work for it, and its bucket is sized to the largest
// contribution:
//
//   1. a rank whose batch is ready (full / timed out / device idle) PROPOSES
//      step k (one compare-and-swap on a shared counter) and rings the bell;
//   2. every rank, when it sees step k proposed and has a free slot, seals its
//      open batch (possibly empty), POSTS the bucket index it needs for step k;
//   3. when all ranks have posted step k, each takes the max bucket and
//      launches step k (identical decision everywhere, no leader round trip).
//
// An idle cluster proposes nothing and launches nothing. The state lives in a
// POSIX shared-memory segment (all ranks of a node map it); waits are futex
// waits on a shared 32-bit bell word with bounded timeouts. Liveness: every
// rank's watcher thread writes a heartbeat (CLOCK_MONOTONIC us); a rank that
// sees a peer silent past the peer timeout marks the segment broken, which
// every rank's server observes and turns into UNAVAILABLE instead of a hang.
//
// This replaces the reference's per-request gRPC fan-out control
// (DCNClient.java:146-164): the data moves over RCCL / the peer kernel, the
// step decision over this segment.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace dtfs {
namespace runtime {

constexpr int kCtlMaxRanks = 64;
constexpr int kCtlRing = 8;  // >= 3 suffices: a rank posts step k only after every rank posted k-1

struct alignas(64) CtlRank {
  std::atomic<uint64_t> post[kCtlRing];  // step k: ((k + 1) << 16) | bucket index
  std::atomic<int64_t> heartbeat_us;      // CLOCK_MONOTONIC microseconds; 0 = not started
  std::atomic<uint32_t> closing;          // this rank stopped admitting and has nothing queued
  std::atomic<uint32_t> attached;
  std::atomic<int32_t> pid;               // the rank's process: a peer whose process is gone is dead at once
  std::atomic<uint64_t> pidns;            // inode of its /proc/self/ns/pid: the pid probe is trusted only within one namespace
};

struct CtlShared {
  uint64_t magic;
  int32_t world;
  uint32_t pad0;
  alignas(64) std::atomic<uint64_t> proposed;  // step k is proposed <=> proposed > k
  // futex words: `bell` wakes idle launchers (through their watcher threads)
  // on a proposal or a state change; `post_bell` wakes ranks gathering a step
  alignas(64) std::atomic<uint32_t> bell;
  std::atomic<uint32_t> waiters;    // threads (any rank) in a futex wait on bell
  std::atomic<uint32_t> idle;       // launchers (any rank) waiting for work: proposals ring only if > 0
  alignas(64) std::atomic<uint32_t> post_bell;
  std::atomic<uint32_t> post_waiters;
  std::atomic<uint32_t> stop;                  // the front door asks every rank to close
  std::atomic<uint32_t> broken;                // sticky: 1 + the rank that gave up first
  std::atomic<uint32_t> epoch;                 // bumped when the cluster is being rebuilt
  alignas(64) CtlRank ranks[kCtlMaxRanks];
};

class StepControl {
 public:
  // create: rank 0 creates (and sizes) the segment; the others attach after it
  // exists (the Python side orders this with a store barrier).
  StepControl(const std::string& name, int world, int rank, bool create);
  ~StepControl();
  StepControl(const StepControl&) = delete;
  StepControl& operator=(const StepControl&) = delete;

  int world() const { return world_; }
  int rank() const { return rank_; }
  const std::string& name() const { return name_; }

  uint64_t proposed() const { return s_->proposed.load(std::memory_order_seq_cst); }
  // Make sure step k is proposed (no-op if someone already did).
  void propose(uint64_t k);
  // This rank's bucket index for step k (call once per step, in step order).
  void post(uint64_t k, int bucket);
  // Wait until every rank posted step k; the agreed bucket (max over ranks),
  // or -1 (timeout, broken, or abort_wait() set) with *err filled.
  int gather(uint64_t k, int64_t timeout_us, std::string* err);

  uint32_t bell() const { return s_->bell.load(std::memory_order_acquire); }
  void ring();
  // Futex wait while bell == seen (bounded). Returns after a ring or timeout.
  void wait_bell(uint32_t seen, int64_t timeout_us) const;
  // This rank's launcher waits for work (proposals ring the bell only while
  // some launcher is idle); seq_cst against propose().
  void set_idle(bool v);

  void heartbeat();
  // First peer whose heartbeat is older than timeout_us (-1: all alive). A peer
  // that never started is judged from `since_us` (this rank's attach time).
  int silent_peer(int64_t timeout_us) const;
  // Microseconds since rank r's last heartbeat (its attach time if it never beat);
  // "forever" once r's process has exited (all ranks of a node share a PID
  // namespace: a dead rank is seen within one watcher period, not after the
  // peer timeout - the peer exchange's readers must stop loading from its store).
  int64_t heartbeat_age_us(int r) const;
  // Rank r's process no longer exists.
  bool process_gone(int r) const;

  void set_closing(bool v);
  bool all_closing() const;
  void request_stop();
  bool stop_requested() const { return s_->stop.load(std::memory_order_acquire) != 0; }
  // Sticky cluster-wide failure flag: returns the rank that broke it (-1: healthy).
  void mark_broken(int by_rank);
  int broken_by() const { return int(s_->broken.load(std::memory_order_acquire)) - 1; }
  uint32_t epoch() const { return s_->epoch.load(std::memory_order_acquire); }
  void bump_epoch();
  // Local: make a thread blocked in gather() return -1 (server shutting down).
  void abort_wait();
  // Remove the segment's name (the mapping stays valid; call after every rank attached).
  void unlink();

 private:
  std::string name_;
  int world_, rank_;
  CtlShared* s_ = nullptr;
  int64_t attach_us_ = 0;
  uint64_t my_pidns_ = 0;  // this process's PID namespace inode (process_gone)
  std::atomic<bool> abort_{false};
};

}  // namespace runtime
}  // namespace dtfs

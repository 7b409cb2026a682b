#include "step_control.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <climits>
#include <cstring>
#include <ctime>
#include <new>
#include <stdexcept>
#include <thread>

#include "batcher.h"  // now_us()

namespace dtfs {
namespace runtime {

namespace {
constexpr uint64_t kMagic = 0x4454465343544c32ull;  // "DTFSCTL2" (CtlRank gained pidns)

// Inode of this process's PID namespace (0 if /proc is not readable).
uint64_t pid_namespace() {
  struct stat st;
  return ::stat("/proc/self/ns/pid", &st) == 0 ? uint64_t(st.st_ino) : 0;
}

uint64_t tag(uint64_t k, int bucket) { return ((k + 1) << 16) | uint64_t(uint16_t(bucket)); }

// Shared (not FUTEX_PRIVATE) futex ops: the word lives in a segment mapped by
// several processes.
void futex_wait(const std::atomic<uint32_t>* w, uint32_t seen, int64_t timeout_us) {
  static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word must be 32 bits");
  timespec ts;
  ts.tv_sec = time_t(timeout_us / 1000000);
  ts.tv_nsec = long(timeout_us % 1000000) * 1000;
  syscall(SYS_futex, reinterpret_cast<const uint32_t*>(w), FUTEX_WAIT, seen, &ts, nullptr, 0);
}

void futex_wake_all(const std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<const uint32_t*>(w), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}
}  // namespace

StepControl::StepControl(const std::string& name, int world, int rank, bool create)
    : name_(name), world_(world), rank_(rank) {
  if (world < 1 || world > kCtlMaxRanks) throw std::invalid_argument("step control: world must be in [1, 64]");
  if (rank < 0 || rank >= world) throw std::invalid_argument("step control: bad rank");
  if (name.empty() || name[0] != '/') throw std::invalid_argument("step control: name must start with '/'");
  const size_t bytes = sizeof(CtlShared);
  int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
  if (create && ftruncate(fd, off_t(bytes)) != 0) {
    const int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error(std::string("ftruncate(step control): ") + std::strerror(e));
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || size_t(st.st_size) < bytes) {
    close(fd);
    throw std::runtime_error("step control segment " + name + " is too small");
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error(std::string("mmap(step control): ") + std::strerror(errno));
  if (create) {
    s_ = new (p) CtlShared();  // value-initialises every atomic to 0
    s_->world = world;
    std::atomic_thread_fence(std::memory_order_release);
    s_->magic = kMagic;
  } else {
    s_ = static_cast<CtlShared*>(p);
    if (s_->magic != kMagic || s_->world != world) {
      munmap(p, bytes);
      throw std::runtime_error("step control segment " + name + " has a different layout or world size");
    }
  }
  attach_us_ = now_us();
  my_pidns_ = pid_namespace();
  s_->ranks[rank_].pidns.store(my_pidns_, std::memory_order_release);
  s_->ranks[rank_].pid.store(int32_t(getpid()), std::memory_order_release);
  s_->ranks[rank_].attached.store(1, std::memory_order_release);
  heartbeat();
}

bool StepControl::process_gone(int r) const {
  if (r < 0 || r >= world_) throw std::out_of_range("step control: rank out of range");
  const int32_t pid = s_->ranks[r].pid.load(std::memory_order_acquire);
  // a pid names the peer only inside the peer's own PID namespace: ranks in
  // other namespaces sharing /dev/shm (sidecar containers) are judged by their
  // heartbeat alone
  const uint64_t ns = s_->ranks[r].pidns.load(std::memory_order_acquire);
  if (pid <= 0 || ns == 0 || ns != my_pidns_) return false;
  return ::kill(pid, 0) != 0 && errno == ESRCH;  // signal 0: existence probe only
}

StepControl::~StepControl() {
  if (s_) munmap(s_, sizeof(CtlShared));
}

void StepControl::ring() {
  s_->bell.fetch_add(1, std::memory_order_seq_cst);
  if (s_->waiters.load(std::memory_order_seq_cst) > 0) futex_wake_all(&s_->bell);
}

namespace {
void ring_posts(CtlShared* s) {
  s->post_bell.fetch_add(1, std::memory_order_seq_cst);
  if (s->post_waiters.load(std::memory_order_seq_cst) > 0) futex_wake_all(&s->post_bell);
}
}  // namespace

void StepControl::set_idle(bool v) {
  if (v) s_->idle.fetch_add(1, std::memory_order_seq_cst);
  else s_->idle.fetch_sub(1, std::memory_order_seq_cst);
}

void StepControl::wait_bell(uint32_t seen, int64_t timeout_us) const {
  if (timeout_us <= 0) return;
  s_->waiters.fetch_add(1, std::memory_order_seq_cst);
  // a ring between the caller's read of `seen` and here has already moved the
  // word, and FUTEX_WAIT returns at once
  futex_wait(&s_->bell, seen, timeout_us);
  s_->waiters.fetch_sub(1, std::memory_order_seq_cst);
}

void StepControl::propose(uint64_t k) {
  uint64_t cur = s_->proposed.load(std::memory_order_seq_cst);
  while (cur <= k && !s_->proposed.compare_exchange_weak(cur, k + 1, std::memory_order_seq_cst)) {
  }
  // an idle launcher (no local work) learns of the step through its watcher;
  // a busy one re-reads `proposed` before it next waits
  if (s_->idle.load(std::memory_order_seq_cst) > 0) ring();
}

void StepControl::post(uint64_t k, int bucket) {
  if (bucket < 0 || bucket > 0xffff) throw std::invalid_argument("step control: bucket index out of range");
  s_->ranks[rank_].post[k % kCtlRing].store(tag(k, bucket), std::memory_order_seq_cst);
  ring_posts(s_);
}

int StepControl::gather(uint64_t k, int64_t timeout_us, std::string* err) {
  const int64_t t0 = now_us();
  const uint64_t want = (k + 1) << 16;
  int spins = 0;
  for (;;) {
    const uint32_t seen = s_->post_bell.load(std::memory_order_seq_cst);
    int best = 0, have = 0;
    for (int r = 0; r < world_; ++r) {
      const uint64_t v = s_->ranks[r].post[k % kCtlRing].load(std::memory_order_acquire);
      if ((v & ~uint64_t(0xffff)) == want) {
        ++have;
        best = std::max(best, int(v & 0xffff));
      }
    }
    if (have == world_) return best;
    const int by = broken_by();
    if (by >= 0) {
      if (err) *err = "cluster broken (rank " + std::to_string(by) + " gave up)";
      return -1;
    }
    if (abort_.load(std::memory_order_acquire)) {
      if (err) *err = "server shutting down";
      return -1;
    }
    const int64_t el = now_us() - t0;
    if (el > timeout_us) {
      if (err) {
        std::string missing;
        for (int r = 0; r < world_; ++r)
          if ((s_->ranks[r].post[k % kCtlRing].load(std::memory_order_acquire) & ~uint64_t(0xffff)) != want)
            missing += (missing.empty() ? "" : ",") + std::to_string(r);
        *err = "step " + std::to_string(k) + ": rank(s) " + missing + " did not join within " +
               std::to_string(el / 1000) + " ms";
      }
      return -1;
    }
    // the other ranks are usually a few microseconds behind: spin briefly
    // before paying for a futex sleep / wake pair
    if (++spins < 64) {
      std::this_thread::yield();
      continue;
    }
    s_->post_waiters.fetch_add(1, std::memory_order_seq_cst);
    futex_wait(&s_->post_bell, seen, std::min<int64_t>(2000, timeout_us - el + 1));
    s_->post_waiters.fetch_sub(1, std::memory_order_seq_cst);
  }
}

void StepControl::heartbeat() { s_->ranks[rank_].heartbeat_us.store(now_us(), std::memory_order_release); }

int64_t StepControl::heartbeat_age_us(int r) const {
  if (r < 0 || r >= world_) throw std::out_of_range("step control: rank out of range");
  if (r != rank_ && process_gone(r)) return INT64_MAX / 4;
  int64_t hb = s_->ranks[r].heartbeat_us.load(std::memory_order_acquire);
  if (hb == 0) hb = attach_us_;
  return now_us() - hb;
}

int StepControl::silent_peer(int64_t timeout_us) const {
  const int64_t now = now_us();
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    if (process_gone(r)) return r;
    int64_t hb = s_->ranks[r].heartbeat_us.load(std::memory_order_acquire);
    if (hb == 0) hb = attach_us_;  // not attached yet: give it the timeout from our start
    if (now - hb > timeout_us) return r;
  }
  return -1;
}

void StepControl::set_closing(bool v) {
  s_->ranks[rank_].closing.store(v ? 1 : 0, std::memory_order_release);
  ring();
}

bool StepControl::all_closing() const {
  for (int r = 0; r < world_; ++r)
    if (!s_->ranks[r].closing.load(std::memory_order_acquire)) return false;
  return true;
}

void StepControl::request_stop() {
  s_->stop.store(1, std::memory_order_release);
  ring();
}

void StepControl::mark_broken(int by_rank) {
  uint32_t expect = 0;
  s_->broken.compare_exchange_strong(expect, uint32_t(by_rank + 1), std::memory_order_acq_rel);
  ring();
  ring_posts(s_);
}

void StepControl::bump_epoch() {
  s_->epoch.fetch_add(1, std::memory_order_acq_rel);
  ring();
}

void StepControl::abort_wait() {
  abort_.store(true, std::memory_order_release);
  ring_posts(s_);
}

void StepControl::unlink() { shm_unlink(name_.c_str()); }

}  // namespace runtime
}  // namespace dtfs

#include "shared_scatter.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <new>
#include <stdexcept>
#include <thread>

#include "arena.h"
#include "batcher.h"  // now_us()
#include "narrow.h"   // kNarrow24Slack
#include "numa.h"

namespace dtfs {
namespace runtime {

namespace {
constexpr uint64_t kMagic = 0x4454465353435431ull;  // "DTFSSCT1"
constexpr int64_t kPage = 4096;
constexpr int64_t kMergeGap = 4096;  // ranges closer than this travel as one copy

int64_t page_up(int64_t x) { return (x + kPage - 1) / kPage * kPage; }

int64_t rd64(const uint8_t* p) {
  int64_t v;
  std::memcpy(&v, p, 8);
  return v;
}
int32_t rd32(const uint8_t* p) {
  int32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// Sorted, merged intervals reduced to at most kShareMaxRanges by closing the
// smallest gaps (a few extra bytes per copy instead of more copies).
int merge_ranges(std::vector<ShareRange>& iv, ShareRange* out) {
  if (iv.empty()) return 0;
  std::sort(iv.begin(), iv.end(), [](const ShareRange& a, const ShareRange& b) { return a.lo < b.lo; });
  std::vector<ShareRange> m;
  m.reserve(iv.size());
  for (const auto& r : iv) {
    if (!m.empty() && r.lo <= m.back().hi + kMergeGap) m.back().hi = std::max(m.back().hi, r.hi);
    else m.push_back(r);
  }
  while (int(m.size()) > kShareMaxRanges) {  // rare: many scattered requests
    size_t best = 1;
    for (size_t i = 2; i < m.size(); ++i)
      if (m[i].lo - m[i - 1].hi < m[best].lo - m[best - 1].hi) best = i;
    m[best - 1].hi = std::max(m[best - 1].hi, m[best].hi);
    m.erase(m.begin() + ptrdiff_t(best));
  }
  for (size_t i = 0; i < m.size(); ++i) out[i] = m[i];
  return int(m.size());
}
}  // namespace

void compute_shares(const uint8_t* arena, int64_t capacity, int64_t fields, int world, int64_t B, RankShare* out) {
  if (world < 1 || world > kScatterMaxRanks || B < 0 || fields < 1) throw std::invalid_argument("compute_shares: bad geometry");
  const int64_t total = rd64(arena + 8);
  const int64_t rt = rd64(arena + 16);
  const int32_t n_chunks = rd32(arena + 32);
  const int32_t wc_hdr = rd32(arena + 36);
  const int32_t idb = rd32(arena + 40) == 3 ? 3 : 4;
  const int64_t payload_cap = capacity - kArenaPayloadOff;
  if (n_chunks > 0) throw std::invalid_argument("shared scatter needs the host varint decode (GPU chunks in the arena)");
  if (total < 0 || total > int64_t(world) * B) throw std::invalid_argument("batch larger than world x rows per rank");
  if (total > 0 && (rt < 0 || rt + 8 * total > payload_cap)) throw std::invalid_argument("row table outside the arena");
  const int64_t wcols = wc_hdr > 0 ? wc_hdr : fields;
  const int32_t* table = reinterpret_cast<const int32_t*>(arena + kArenaPayloadOff + rt);
  std::vector<ShareRange> iv;
  // even split on row boundaries (the reference splits every request's
  // candidates over all shards, DCNClient.java:46-74): a partial batch still
  // spreads over every GPU's link; each share fits the bucket (<= B rows)
  const int64_t per = (total + world - 1) / world;
  for (int r = 0; r < world; ++r) {
    RankShare& s = out[r];
    s = RankShare();
    s.row0 = std::min(total, int64_t(r) * per);
    s.rows = std::max<int64_t>(0, std::min(total, s.row0 + per) - s.row0);
    iv.clear();
    int64_t last_ids = -1, last_wts = -1;  // the interval each stream extends
    auto add = [&](int64_t lo, int64_t n, int64_t& last) {
      const int64_t hi = std::min(payload_cap, lo + n);
      lo = std::max<int64_t>(0, lo);
      if (hi <= lo) return;
      if (last >= 0 && lo >= iv[size_t(last)].lo && lo <= iv[size_t(last)].hi + kMergeGap) {
        iv[size_t(last)].hi = std::max(iv[size_t(last)].hi, hi);
        return;
      }
      iv.push_back(ShareRange{lo, hi});
      last = int64_t(iv.size()) - 1;
    };
    for (int64_t i = s.row0; i < s.row0 + s.rows; ++i) {
      const int32_t x = table[2 * i], y = table[2 * i + 1];
      const bool narrow = x < 0;
      const int64_t ids_off = int64_t(uint32_t(x) & 0x7fffffffu);
      add(ids_off, narrow ? idb * fields + kNarrow24Slack : 8 * fields, last_ids);
      if (narrow) {  // weights of kind y >> 30 (none for all-ones requests)
        const int64_t wb = wts_bytes_per(int(uint32_t(y) >> kWtsKindShift)) * wcols;
        if (wb > 0) add(int64_t(uint32_t(y) & ((1u << kWtsKindShift) - 1)), wb, last_wts);
      } else {
        add(int64_t(y), 4 * fields, last_wts);
      }
    }
    s.n_ranges = merge_ranges(iv, s.r);
  }
}

std::vector<ShareCopy> share_copies(const uint8_t* arena, const RankShare& s, uint8_t* hdr_stage) {
  std::memcpy(hdr_stage, arena, 64);
  const int64_t rows = s.rows;
  std::memcpy(hdr_stage + 8, &rows, 8);
  const int32_t zero = 0;
  std::memcpy(hdr_stage + 32, &zero, 4);  // no GPU varint chunks
  const int64_t rt = rd64(arena + 16);
  std::vector<ShareCopy> c;
  c.reserve(size_t(2 + s.n_ranges));
  c.push_back(ShareCopy{0, hdr_stage, 64});
  if (rows > 0) {
    // this rank's rows of the row table, moved to the table's start (row i of
    // the share is row 0 + i of the device arena)
    c.push_back(ShareCopy{kArenaPayloadOff + rt, arena + kArenaPayloadOff + rt + 8 * s.row0, 8 * rows});
    for (int i = 0; i < s.n_ranges; ++i)
      c.push_back(ShareCopy{kArenaPayloadOff + s.r[i].lo, arena + kArenaPayloadOff + s.r[i].lo, s.r[i].hi - s.r[i].lo});
  }
  return c;
}

std::vector<NodeSlice> scatter_placement(int64_t arenas_off, int n_arenas, int64_t arena_stride, int64_t payload_off,
                                         int64_t expected_payload, const std::vector<int>& rank_nodes) {
  std::vector<NodeSlice> out;
  const int world = int(rank_nodes.size());
  if (world < 2 || expected_payload <= 0 || n_arenas < 1) return out;
  const int64_t cap = arena_stride - payload_off;  // payload bytes an arena can hold
  const int64_t used = std::min(expected_payload, cap);
  for (int i = 0; i < n_arenas; ++i) {
    const int64_t p0 = arenas_off + int64_t(i) * arena_stride + payload_off;
    for (int r = 1; r < world; ++r) {
      const int nd = rank_nodes[size_t(r)];
      if (nd < 0 || nd == rank_nodes[0]) continue;  // rank 0's node already holds the segment
      // whole pages only: the boundary page stays with the lower share
      int64_t lo = page_up(p0 + used * r / world);
      int64_t hi = r == world - 1 ? arenas_off + int64_t(i + 1) * arena_stride : page_up(p0 + used * (r + 1) / world);
      hi = std::min(hi, arenas_off + int64_t(i + 1) * arena_stride);
      if (hi <= lo) continue;
      if (!out.empty() && out.back().node == nd && out.back().hi == lo) out.back().hi = hi;  // neighbours on one node
      else out.push_back(NodeSlice{lo, hi, nd, r, false});
    }
  }
  return out;
}

SharedScatter::SharedScatter(const std::string& name, int world, int rank, bool create, int64_t fields, int n_arenas,
                             int64_t arena_cap, int slots, int64_t out_floats, int node,
                             const std::vector<int>& rank_nodes, int64_t expected_payload)
    : name_(name), rank_(rank) {
  if (world < 1 || world > kScatterMaxRanks) throw std::invalid_argument("shared scatter: world must be in [1, 16]");
  if (rank < 0 || rank >= world) throw std::invalid_argument("shared scatter: bad rank");
  if (name.empty() || name[0] != '/') throw std::invalid_argument("shared scatter: name must start with '/'");
  const int64_t hdr = page_up(int64_t(sizeof(ScatterShared)));
  int64_t arenas_off = 0, outs_off = 0, total = 0;
  if (create) {
    if (n_arenas < 1 || arena_cap <= kArenaPayloadOff || slots < 1 || slots > kScatterMaxSlots || out_floats < 1 ||
        fields < 1)
      throw std::invalid_argument("shared scatter: bad segment geometry");
    arenas_off = hdr;
    outs_off = arenas_off + int64_t(n_arenas) * page_up(arena_cap);
    total = outs_off + int64_t(slots) * page_up(out_floats * 4);
  }
  int fd = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
  if (create && ftruncate(fd, off_t(total)) != 0) {
    const int e = errno;
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error(std::string("ftruncate(shared scatter): ") + std::strerror(e));
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < off_t(hdr)) {
    close(fd);
    throw std::runtime_error("shared scatter segment " + name + " is too small");
  }
  bytes_ = size_t(st.st_size);
  void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (create) shm_unlink(name.c_str());
    throw std::runtime_error(std::string("mmap(shared scatter): ") + std::strerror(errno));
  }
  base_ = static_cast<uint8_t*>(p);
  if (create) {
    // rank 0 writes every request into these pages: place them on its node
    // before anything touches them (best effort)
    if (node >= 0) bind_range_to_node(p, bytes_, node);
    if (!rank_nodes.empty()) {
      if (int(rank_nodes.size()) != world) {
        munmap(p, bytes_);
        shm_unlink(name.c_str());
        throw std::invalid_argument("shared scatter: rank_nodes needs one node per rank");
      }
      // then each rank's share of every arena on that rank's node (before
      // anything touches the pages; best effort like the segment's own)
      placement_ = scatter_placement(arenas_off, n_arenas, page_up(arena_cap), kArenaPayloadOff, expected_payload,
                                     rank_nodes);
      for (auto& sl : placement_) sl.bound = bind_range_to_node(static_cast<uint8_t*>(p) + sl.lo, size_t(sl.hi - sl.lo), sl.node);
    }
    s_ = new (p) ScatterShared();
    s_->world = world;
    s_->n_arenas = n_arenas;
    s_->slots = slots;
    s_->fields = fields;
    s_->arena_cap = arena_cap;
    s_->out_floats = out_floats;
    s_->arenas_off = arenas_off;
    s_->outs_off = outs_off;
    s_->total_bytes = total;
    std::atomic_thread_fence(std::memory_order_release);
    s_->magic = kMagic;
  } else {
    s_ = reinterpret_cast<ScatterShared*>(p);
    if (s_->magic != kMagic || s_->world != world || int64_t(bytes_) < s_->total_bytes) {
      munmap(p, bytes_);
      throw std::runtime_error("shared scatter segment " + name + " has a different layout or world size");
    }
  }
  s_->attached[rank_].store(1, std::memory_order_release);
}

SharedScatter::~SharedScatter() {
  if (!base_) return;
  if (on_unmap_) on_unmap_(base_, bytes_);
  munmap(base_, bytes_);
}

uint8_t* SharedScatter::stage(int slot) const {
  if (slot < 0 || slot >= kScatterMaxSlots) throw std::out_of_range("shared scatter: slot beyond the header stages");
  return s_->stage[rank_][slot];
}

uint8_t* SharedScatter::arena(int i) const {
  if (i < 0 || i >= s_->n_arenas) throw std::out_of_range("shared scatter: arena index");
  return base_ + s_->arenas_off + int64_t(i) * page_up(s_->arena_cap);
}

float* SharedScatter::out(int slot) const {
  if (slot < 0 || slot >= s_->slots) throw std::out_of_range("shared scatter: slot");
  return reinterpret_cast<float*>(base_ + s_->outs_off + int64_t(slot) * page_up(s_->out_floats * 4));
}

int SharedScatter::arena_index(const uint8_t* p) const {
  for (int i = 0; i < s_->n_arenas; ++i)
    if (arena(i) == p) return i;
  return -1;
}

bool SharedScatter::all_attached() const {
  for (int r = 0; r < s_->world; ++r)
    if (!s_->attached[r].load(std::memory_order_acquire)) return false;
  return true;
}

void SharedScatter::unlink() { shm_unlink(name_.c_str()); }

void SharedScatter::publish_plan(uint64_t k, int arena_idx, int64_t rows_per_rank) {
  if (rank_ != 0) throw std::logic_error("shared scatter: only rank 0 publishes plans");
  StepPlan& P = s_->plans[k % kPlanRing];
  P.seq.store(0, std::memory_order_relaxed);
  P.arena = arena_idx;
  P.world = s_->world;
  P.rows_per_rank = rows_per_rank;
  const uint8_t* a = arena(arena_idx);
  P.total_rows = rd64(a + 8);
  compute_shares(a, s_->arena_cap, s_->fields, s_->world, rows_per_rank, P.share);
  P.seq.store(k + 1, std::memory_order_release);
}

bool SharedScatter::wait_plan(uint64_t k, int64_t timeout_us, RankShare* mine, int* arena_idx) {
  const StepPlan& P = s_->plans[k % kPlanRing];
  const int64_t t0 = now_us();
  for (int spins = 0;; ++spins) {
    if (P.seq.load(std::memory_order_acquire) == k + 1) break;
    if (now_us() - t0 > timeout_us) return false;
    if (spins < 4000) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  *mine = P.share[rank_];
  *arena_idx = P.arena;
  return true;
}

void SharedScatter::compact_scores(uint64_t k, int slot) {
  // rank r's step wrote its rows' scores at r * rows_per_rank (the captured
  // head's fixed slice); the batch reads row j at j: move each share down to
  // its first row (ascending ranks: destinations never pass their sources)
  const StepPlan& P = s_->plans[k % kPlanRing];
  if (P.seq.load(std::memory_order_acquire) != k + 1) throw std::logic_error("shared scatter: plan overwritten");
  float* o = out(slot);
  for (int r = 1; r < P.world; ++r) {
    const RankShare& sh = P.share[r];
    const int64_t src = int64_t(r) * P.rows_per_rank;
    if (sh.rows > 0 && sh.row0 != src) {
      if (src + sh.rows > s_->out_floats) throw std::out_of_range("shared scatter: share outside the output");
      std::memmove(o + sh.row0, o + src, size_t(sh.rows) * sizeof(float));
    }
  }
}

void SharedScatter::mark_done(uint64_t k) { s_->done[rank_].store(k + 1, std::memory_order_release); }

bool SharedScatter::wait_done(uint64_t k, int64_t timeout_us, std::string* err) const {
  const int64_t t0 = now_us();
  for (int r = 0; r < s_->world; ++r) {
    for (int spins = 0; s_->done[r].load(std::memory_order_acquire) < k + 1; ++spins) {
      if (now_us() - t0 > timeout_us) {
        if (err)
          *err = "rank " + std::to_string(r) + " did not finish its share of step " + std::to_string(k) + " within " +
                 std::to_string(timeout_us / 1000) + " ms";
        return false;
      }
      if (spins < 4000) std::this_thread::yield();
      else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  return true;
}

}  // namespace runtime
}  // namespace dtfs

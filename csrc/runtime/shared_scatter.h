// Scatter fan-out through shared host memory instead of a device collective.
//
// In scatter mode rank 0 is the only front door (the reference topology,
// DCNClient.java:146-164: one client splits every request over the shards).
// With an RCCL scatter, rank 0's ONE PCIe link carries every rank's request
// bytes and then xGMI moves them again. Here rank 0's request arenas and its
// score outputs live in one POSIX shared-memory segment that every rank of the
// node maps (and registers with its own GPU). Per step k:
//
//   rank 0   builds its batch (world x B rows) in a shared arena, then
//            publishes the step's PLAN: for every rank r its rows
//            [r B, r B + rows_r) and the few payload byte ranges those rows read
//            (from the arena's row table; requests are appended in order, so a
//            share is one or two ranges)
//   rank r   reads the plan and DMAs only its share over its OWN PCIe link
//            into a device arena of the same layout: a patched 64-byte header
//            (total_rows = rows_r) from private pinned memory, its slice of the
//            row table moved to the table's start, and its payload ranges at
//            their own offsets - so the unmodified local step kernels run on it
//            and the head writes rank r's scores straight into rank 0's shared
//            output at r B; then it reports step k done in the segment
//   rank 0   answers step k once every rank reported it (bounded wait)
//
// Host->device bytes per rank: its share, not the whole batch; nothing crosses
// xGMI. The RCCL scatter (parallel/fanout.py) stays the fallback (different
// nodes, or a segment that cannot be registered).
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace dtfs {
namespace runtime {

constexpr int kScatterMaxRanks = 16;
constexpr int kShareMaxRanges = 8;
constexpr int kPlanRing = 16;  // > slots: rank 0 can run at most `slots` steps ahead of a follower
constexpr int kScatterMaxSlots = 8;

struct ShareRange {
  int64_t lo = 0, hi = 0;  // payload-relative [lo, hi)
};

struct RankShare {
  int64_t row0 = 0, rows = 0;
  int32_t n_ranges = 0;
  int32_t pad = 0;
  ShareRange r[kShareMaxRanges];
};

struct alignas(64) StepPlan {
  std::atomic<uint64_t> seq;  // k + 1 once the plan of step k is complete
  int32_t arena;              // index of the shared arena holding the batch
  int32_t world;
  int64_t total_rows, rows_per_rank;
  RankShare share[kScatterMaxRanks];
};

struct alignas(64) ScatterShared {
  uint64_t magic;
  int32_t world, n_arenas, slots, pad0;
  int64_t fields, arena_cap, out_floats, arenas_off, outs_off, total_bytes;
  alignas(64) std::atomic<uint64_t> done[kScatterMaxRanks];  // steps [0, done) finished on rank r
  std::atomic<uint32_t> attached[kScatterMaxRanks];
  StepPlan plans[kPlanRing];
  // per (rank, slot): the patched 64-byte arena header a rank copies to its
  // device (in the segment so that the GPU registration covers it)
  alignas(64) uint8_t stage[kScatterMaxRanks][kScatterMaxSlots][64];
};

// One copy of a rank's share: `n` bytes from host `src` to device arena offset `dst_off`.
struct ShareCopy {
  int64_t dst_off;
  const uint8_t* src;
  int64_t n;
};

// Rank shares of a built arena (`arena`: its base; header + row table parsed
// here): rows split evenly on row boundaries (ceil(total / world) per rank,
// <= B) and the merged payload ranges they read.
// `fields`: features per row (the row spans' sizes). Throws when the arena
// defers ids to the GPU varint decode (its row table then points past the
// copied bytes).
void compute_shares(const uint8_t* arena, int64_t capacity, int64_t fields, int world, int64_t rows_per_rank,
                    RankShare* out);
// The copies that bring `s` of `arena` into a device arena of the same layout.
// `hdr_stage`: 64 bytes of this rank's pinned memory that receive the patched
// header (total_rows = s.rows, GPU varint decode off).
std::vector<ShareCopy> share_copies(const uint8_t* arena, const RankShare& s, uint8_t* hdr_stage);

// NUMA placement of the shared arenas, per rank: requests are appended in row
// order and shares are contiguous row ranges, so rank r's bytes of a full batch
// sit at about payload [r S, (r + 1) S), S = expected_payload / world. Those
// pages go on the NUMA node of the GPU that DMAs them (rank 0's thread writes
// them once across the socket link instead of that GPU reading them across it
// every step). Byte offsets are segment-relative, page-aligned.
struct NodeSlice {
  int64_t lo = 0, hi = 0;
  int node = -1;
  int rank = -1;
  bool bound = false;  // mbind succeeded (false: one-node machine / no NUMA support)
};
std::vector<NodeSlice> scatter_placement(int64_t arenas_off, int n_arenas, int64_t arena_stride, int64_t payload_off,
                                         int64_t expected_payload, const std::vector<int>& rank_nodes);

class SharedScatter {
 public:
  // create (rank 0): the segment sized for n_arenas arenas of arena_cap bytes
  // and `slots` outputs of out_floats fp32 scores; node >= 0 places its pages
  // on that NUMA node, then rank_nodes (one node per rank, -1 unknown) and
  // expected_payload (bytes of a full batch) place each rank's share of every
  // arena on its own node (scatter_placement). attach (rank > 0): map an
  // existing segment.
  SharedScatter(const std::string& name, int world, int rank, bool create, int64_t fields = 0, int n_arenas = 0,
                int64_t arena_cap = 0, int slots = 0, int64_t out_floats = 0, int node = -1,
                const std::vector<int>& rank_nodes = {}, int64_t expected_payload = 0);
  ~SharedScatter();
  SharedScatter(const SharedScatter&) = delete;
  SharedScatter& operator=(const SharedScatter&) = delete;

  int world() const { return s_->world; }
  int rank() const { return rank_; }
  int n_arenas() const { return s_->n_arenas; }
  int slots() const { return s_->slots; }
  int64_t arena_cap() const { return s_->arena_cap; }
  int64_t fields() const { return s_->fields; }
  int64_t out_floats() const { return s_->out_floats; }
  uint8_t* arena(int i) const;
  float* out(int slot) const;
  int arena_index(const uint8_t* base) const;  // -1: not one of the segment's arenas
  uint8_t* stage(int slot) const;              // this rank's header stage of a slot
  void* base() const { return base_; }
  size_t bytes() const { return bytes_; }
  // called with (base, bytes) before the mapping goes away (e.g. hipHostUnregister)
  void set_on_unmap(std::function<void(void*, size_t)> f) { on_unmap_ = std::move(f); }
  bool all_attached() const;
  void unlink();
  // create side: the per-rank slices placed at creation (empty on attach)
  const std::vector<NodeSlice>& placement() const { return placement_; }

  // The step index of the next launch on this rank (every rank launches every
  // step in the same order, so the counters agree).
  uint64_t begin_step() { return next_step_++; }
  // Rank 0: the plan of step k over the built arena `arena_idx`.
  void publish_plan(uint64_t k, int arena_idx, int64_t rows_per_rank);
  // The plan of step k (false: not published within timeout_us).
  bool wait_plan(uint64_t k, int64_t timeout_us, RankShare* mine, int* arena_idx);
  // Rank 0, once every rank finished step k on `slot`: move each rank's
  // scores from its fixed slice (r x rows_per_rank) to its rows' place.
  void compact_scores(uint64_t k, int slot);
  // This rank finished step k (its scores are in the shared output).
  void mark_done(uint64_t k);
  // Every rank finished step k (false after timeout_us; *err names the late rank).
  bool wait_done(uint64_t k, int64_t timeout_us, std::string* err) const;

  // Accounting: host->device bytes this rank copied for its shares.
  void add_h2d(int64_t n) { h2d_bytes_.fetch_add(n, std::memory_order_relaxed); h2d_steps_.fetch_add(1, std::memory_order_relaxed); }
  int64_t h2d_bytes() const { return h2d_bytes_.load(); }
  int64_t h2d_steps() const { return h2d_steps_.load(); }

 private:
  std::string name_;
  int rank_;
  size_t bytes_ = 0;
  ScatterShared* s_ = nullptr;
  uint8_t* base_ = nullptr;
  std::atomic<uint64_t> next_step_{0};
  std::atomic<int64_t> h2d_bytes_{0}, h2d_steps_{0};
  std::function<void(void*, size_t)> on_unmap_;
  std::vector<NodeSlice> placement_;
};

}  // namespace runtime
}  // namespace dtfs

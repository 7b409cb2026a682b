// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave = 64 lanes (never 32); block sizes are multiples of 64.
//   * bf16 tensors are moved 16 bytes per lane (8 x bf16) - hipcc does not
//     vectorise scalar bf16 loads on its own.
//   * matrices are row-major with the reduction dim contiguous: activations
//     [M][K], weights [N][K] (torch Linear layout), so both MFMA operands are
//     16-byte contiguous runs per lane.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtfs {
namespace kern {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return float(x); }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// v_rcp_f32 (1 ulp) instead of an IEEE division: the division's div_scale /
// div_fmas / div_fixup sequence is ~10 instructions per element in unrolled
// epilogues. exp(-x) = inf -> 0, exp(-x) = 0 -> 1 as before.
__device__ __forceinline__ float sigmoidf(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// Hash an incoming feature id onto a table row (K0 semantics): python-style
// non-negative modulo; modulo <= 0 means ids are already row indices.
__device__ __forceinline__ int64_t hash_row(int64_t id, int64_t modulo) {
  if (modulo <= 0) return id;
  int64_t r = id % modulo;
  return r < 0 ? r + modulo : r;
}

// u mod m for m < 2^32 with magic = floor((2^64 - 1) / m): q = mulhi(u, magic)
// is floor(u/m) or one less, so one conditional subtract finishes it (the
// 64-bit software modulo of hash_row costs ~100 instructions).
__device__ __forceinline__ int64_t hash_row_magic(int64_t id, int64_t m, uint64_t magic) {
  const uint64_t u = id < 0 ? uint64_t(0) - uint64_t(id) : uint64_t(id);
  const uint64_t q = __umul64hi(u, magic);
  uint64_t r = u - q * uint64_t(m);
  if (r >= uint64_t(m)) r -= uint64_t(m);
  if (id < 0 && r) r = uint64_t(m) - r;  // python-style non-negative modulo
  return int64_t(r);
}

// Unaligned little-endian loads from byte-addressed buffers (protobuf
// tensor_content has no alignment): aligned dword loads + v_alignbyte funnel
// shifts instead of byte loads. Reads only the dwords the value overlaps.
__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const int sh = int(a & 3);
  const uint32_t w0 = w[0], w1 = w[1];
  const uint32_t w2 = sh ? w[2] : 0u;
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return (uint64_t(hi) << 32) | lo;
}

__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const int sh = int(a & 3);
  const uint32_t w0 = w[0];
  const uint32_t w1 = sh ? w[1] : 0u;
  return __builtin_amdgcn_alignbyte(w1, w0, sh);
}

// Request-arena header (csrc/runtime/arena.h): n_req @0, total_rows @8,
// row_table_off @16 ({ids_off, wts_off} int32 per row, payload-relative).
// A row whose ids_off has bit 31 set was narrowed by the host while it copied
// the request (runtime/narrow.h): int32 table rows + fp32 weights, aligned.
// Header @36 (int32 narrow_wcols): > 0 = a narrowed row carries only its
// first narrow_wcols weights (the model reads no others); the rest read as 0.
constexpr int kArenaAllWeights = 1 << 30;
__device__ __forceinline__ int arena_narrow_wcols(const uint8_t* arena) {
  const int w = *reinterpret_cast<const int32_t*>(arena + 36);
  return w > 0 ? w : kArenaAllWeights;
}

// Header @40 (int32): 3 = narrowed rows hold packed 3-byte table rows.
__device__ __forceinline__ int arena_narrow_idb(const uint8_t* arena) {
  return *reinterpret_cast<const int32_t*>(arena + 40) == 3 ? 3 : 4;
}

// Row-table wts_off of a narrowed row, bits 31..30: how its weights travel
// (runtime/narrow.h WtsKind): fp32, bf16 (every weight of the request was
// exactly a bf16 value) or none (every weight was 1.0, the reference client's
// requests, DCNClient.java:67-73). Bits 29..0: the payload offset.
constexpr uint32_t kWtsOffMask = 0x3fffffffu;
constexpr int kWtsF32 = 0, kWtsBf16 = 1, kWtsOnes = 2;

struct ArenaRow {
  const uint8_t* ids;  // 8 * F bytes of int64 ids (narrow: idb * F bytes of rows), or nullptr (padding row)
  const uint8_t* wts;  // 4 * F bytes of fp32 weights (narrow: wcols weights of kind wkind)
  bool narrow;
  int wcols;  // narrow rows: weights present (arena_narrow_wcols)
  int idb;    // narrow rows: bytes per id (arena_narrow_idb)
  int wkind = kWtsF32;  // narrow rows: kWtsF32 / kWtsBf16 / kWtsOnes
};

// Table row of feature f of a narrowed row: int32, or 3 packed bytes (the
// 4-byte load of the last one stays inside the arena's slack)
__device__ __forceinline__ int64_t arena_narrow_id(const ArenaRow& ar, int f) {
  if (ar.idb == 3) return int64_t(load_u32_unaligned(ar.ids + 3 * f) & 0xffffffu);
  return int64_t(reinterpret_cast<const int32_t*>(ar.ids)[f]);
}

// Weight f of a narrowed row (0 past the columns the row carries).
__device__ __forceinline__ float arena_narrow_w(const ArenaRow& ar, int f) {
  if (f >= ar.wcols) return 0.f;
  if (ar.wkind == kWtsOnes) return 1.f;
  if (ar.wkind == kWtsBf16) return __uint_as_float(uint32_t(reinterpret_cast<const uint16_t*>(ar.wts)[f]) << 16);
  return reinterpret_cast<const float*>(ar.wts)[f];
}

// A row-table entry {ids_off, wts_off} of the payload -> the row.
__device__ __forceinline__ ArenaRow arena_row_at(const uint8_t* payload, int2 o, int wcols, int idb) {
  ArenaRow r{payload + (o.x & 0x7fffffff), payload + (uint32_t(o.y) & kWtsOffMask), o.x < 0, kArenaAllWeights, 4};
  if (r.narrow) {
    r.wcols = wcols;
    r.idb = idb;
    r.wkind = int(uint32_t(o.y) >> 30);
  }
  return r;
}

__device__ __forceinline__ ArenaRow arena_row(const uint8_t* arena, int64_t payload_off, int64_t r) {
  const int64_t total = *reinterpret_cast<const int64_t*>(arena + 8);
  ArenaRow out{nullptr, nullptr, false, kArenaAllWeights, 4};
  if (r < total) {
    const uint8_t* payload = arena + payload_off;
    const int64_t rt = *reinterpret_cast<const int64_t*>(arena + 16);
    const int2 o = reinterpret_cast<const int2*>(payload + rt)[r];
    out = arena_row_at(payload, o, arena_narrow_wcols(arena), arena_narrow_idb(arena));
  }
  return out;
}

// Feature f of an arena row: raw int64 id (narrow: int32 row) and fp32 weight.
__device__ __forceinline__ void arena_feature(const ArenaRow& ar, int f, int64_t& id, float& w) {
  if (ar.narrow) {
    id = arena_narrow_id(ar, f);
    w = arena_narrow_w(ar, f);
  } else {
    id = int64_t(load_u64_unaligned(ar.ids + 8 * f));
    w = __uint_as_float(load_u32_unaligned(ar.wts + 4 * f));
  }
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks b and b+8 share an XCD under the
// observed round-robin dispatch, so give each XCD a contiguous run of tiles so
// neighbouring tiles (which share operand panels) hit the same L2. Speed only;
// correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return orig;
  const int q = nwg / NX, r = nwg % NX;
  const int xcd = orig % NX, slot = orig / NX;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + slot;
}

}  // namespace kern
}  // namespace dtfs

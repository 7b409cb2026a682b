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

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

// Hash an incoming feature id onto a table row (K0 semantics): python-style
// non-negative modulo; modulo <= 0 means ids are already row indices.
__device__ __forceinline__ int64_t hash_row(int64_t id, int64_t modulo) {
  if (modulo <= 0) return id;
  int64_t r = id % modulo;
  return r < 0 ? r + modulo : r;
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

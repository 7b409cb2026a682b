// Inline-asm memory operations for hand-scheduled gfx950 loops.
//
// The kernels that keep several K tiles in flight (mlp_tail.hip,
// gather_gemm.hip) issue their LDS-DMA, register loads and LDS reads through
// these wrappers and place every s_waitcnt themselves:
//   * with __builtin_amdgcn_global_load_lds, the waitcnt pass puts a vmcnt(0)
//     in front of MFMAs whose operands came from ordinary global loads (the
//     LDS-DMA's pending event merges with them; gfx950 ISA, ROCm 7.2), which
//     drains a prefetch every K tile;
//   * ds_reads of a ring the DMA writes get a vmcnt(0) in front of them too
//     (LDS alias tracking).
// Contract: a value produced by lds_read16 / gload16 may be used only after a
// wait_* call that names it as an operand ("+v"), so the compiler cannot move
// its use above the wait. The caller computes the counts: vmcnt / lgkmcnt
// retire in issue order.
#pragma once

#include "common.h"

namespace dtfs {
namespace kern {

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}

// 16 bytes per lane global -> LDS (lane i lands at lds + 16 i); M0 holds the
// wave-uniform LDS base.
__device__ __forceinline__ void lds_dma16(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
}

__device__ __forceinline__ bf16x8 lds_read16(const uint8_t* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}

__device__ __forceinline__ i32x4 lds_read16i(const uint8_t* p) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}

__device__ __forceinline__ int lds_read4(const void* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}

__device__ __forceinline__ void lds_write16(uint8_t* p, const i32x4& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}

// SGPR base + 32-bit per-lane byte offset: the uniform part of an address
// stays in scalar registers (no 64-bit VALU adds, one VGPR per address)
__device__ __forceinline__ void lds_dma16_s(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory", "m0");
}

// 4 bytes per lane into LDS at M0 + 4 lane: a cache-line touch with no
// register destination (nothing for the compiler to reuse while it is in flight)
__device__ __forceinline__ void lds_dma4_s(const void* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory", "m0");
}

__device__ __forceinline__ bf16x8 gload16_s(const void* sbase, uint32_t voff) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(v) : "v"(voff), "s"(sbase));
  return v;
}

// 16 bytes per lane global -> registers
__device__ __forceinline__ bf16x8 gload16(const void* g) {
  bf16x8 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(g));
  return v;
}

}  // namespace kern
}  // namespace dtfs

// K4 + K4 + K6 fused: the MLP tail of DeepFM / Wide&Deep / DCN (SURVEY §2.4
// K4 "mlp_tower" + K6 "head_sigmoid") in one launch:
//
//   h2 = act2(X W2^T + b2)             [M, N2]  bf16, kept in LDS
//   h3 = act3(h2 W3^T + b3)            [M, N3]  fp32, kept in registers
//   y[m] = out_act(h3[m, :] . hw + hbias + sum_e extra[e][m])
//
// The served step used to run this as GEMM2 (128x128 tiles, h2 through HBM)
// + the fused last-layer/head kernel: 22.6 + 10-14 us at 16384 rows, both
// far from the matrix cores' rate (0.76 PF and ~0.4 PF), plus one kernel
// boundary. Here one 512-thread workgroup owns 64 rows (16384 rows = 256
// workgroups, one per CU) and runs both GEMMs back to back:
//
//   * A (X rows, 64 x K1) is the only operand shared by the 8 waves: it goes
//     through a 4-slot LDS ring of 64-deep K tiles (8 KiB each), one LDS-DMA
//     instruction per wave per tile, issued two tiles ahead; one s_barrier
//     per K tile.
//   * B (W2 / W3) is private to each wave (wave w owns output columns
//     [w N/8, (w+1) N/8)), so it never touches LDS: the weights are kept in
//     MFMA fragment order (pack_bfrag: every wave-instruction reads 1 KiB of
//     contiguous bytes) and loaded straight into registers one K tile ahead.
//   * h2 (64 x 512 bf16 = 64 KiB) is written to LDS by the GEMM2 epilogue
//     (bias + ReLU + bf16, the unfused path's rounding) with a 16-byte chunk
//     XOR swizzle by row, and read back as GEMM3's A operand.
//   * the head reduces h3 . hw per row across lanes and waves in LDS and
//     writes one score per row (device or mapped pinned-host memory).
//
// MFMA: v_mfma_f32_16x16x32_bf16 in the transposed form used by every GEMM
// here (D = W_frag x A_frag^T: lane (fr, fq) holds C[m = fr][n = 4 fq .. +3]).
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

// Ablations for tools/native/tail_ablate.hip only (wrong results): bit 0
// drops GEMM2's B loads in the K loop, 1 its A DMAs, 2 the per-tile barrier,
// 3 GEMM3 and the head.
#ifndef TAIL_ABL
#define TAIL_ABL 0
#endif

namespace {
// A ring tile: 64 rows x 128 bytes, 16-byte chunk c of row r at c ^ ((r >> 1) & 7)
__device__ __forceinline__ int tail_swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// A fragment read from the ring as inline asm: the compiler cannot tell these
// reads from the in-flight LDS-DMA writes of other ring slots and otherwise
// puts a vmcnt(0) in front of them (draining the B prefetch every other K
// tile, gfx950 ISA). The caller waits lgkmcnt itself, with the fragments as
// in/out operands of that wait so no MFMA is scheduled above it.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}
// 16 bytes per lane global -> LDS (lane i lands at lds + 16 i), as inline asm:
// with the builtin, the waitcnt pass drains every in-flight load (vmcnt(0))
// before the MFMAs that use register-loaded B fragments (gfx950 ISA). M0
// carries the wave-uniform LDS base.
__device__ __forceinline__ void lds_dma16(const void* g, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ bf16x8 lds_read16(const uint8_t* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}
}  // namespace

template <int K1, int N2, int N3>
__global__ void __launch_bounds__(512) mlp_tail_kernel(const bf16* __restrict__ X, int64_t ldx, int M,
                                                       const bf16x8* __restrict__ W2p, const float* __restrict__ b2,
                                                       int act2, const bf16x8* __restrict__ W3p,
                                                       const float* __restrict__ b3, int act3,
                                                       const float* __restrict__ hw, float hbias,
                                                       const float* __restrict__ extra, int extra_n, int64_t extra_ld,
                                                       int out_act, float* __restrict__ y) {
  constexpr int BM = 64, NW = 8;
  constexpr int NS = 4, LEAD = 2;  // ring slots; tiles DMA'd ahead (NS >= LEAD + 2: see the WAR note below)
  constexpr int SLOT = BM * 128;
  constexpr int H2P = N2 * 2;     // h2 row pitch (bytes)
  constexpr int TJ2 = N2 / NW / 16;  // 16-column blocks per wave, GEMM2
  constexpr int TJ3 = N3 / NW / 16;  // GEMM3
  constexpr int NK2 = N2 / 64;       // GEMM3 K tiles
  static_assert(N2 % (16 * NW) == 0 && N3 % (16 * NW) == 0 && NK2 % 2 == 0, "tail shape");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * SLOT + BM * H2P + NW * BM * 4];
  uint8_t* ring = smem;
  uint8_t* h2s = smem + NS * SLOT;
  float* red = reinterpret_cast<float*>(h2s + BM * H2P);

  const int m0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int nkt = K1 / 64;

  // A staging: wave wid DMAs rows 8 wid .. 8 wid + 7 of every K tile (1 KiB;
  // lane i lands at +16 i, so its source is the logical chunk that swizzles there)
  const int ar = 8 * wid + (lane >> 3);
  const bf16* a_src = X + int64_t(min(m0 + ar, M - 1)) * ldx + (((lane & 7) ^ ((ar >> 1) & 7)) << 3);
  const uint32_t ring_lds = lds_addr(ring) + wid * 1024;
  auto stage_a = [&](int kt) {
    const int kc = min(kt, nkt - 1);  // trailing stages re-load the last tile (branch-free loop)
    lds_dma16(a_src + kc * 64, ring_lds + (kt % NS) * SLOT);
  };
  // B fragments of this wave's columns: packed block jb = wid * TJ + j
  const bf16x8* w2w = W2p + int64_t(wid * TJ2) * nkt * 2 * 64 + lane;
  auto load_b2 = [&](bf16x8(&b)[TJ2][2], int kt) {
    const int kc = min(kt, nkt - 1);
#pragma unroll
    for (int j = 0; j < TJ2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b[j][kk] = w2w[((j * nkt + kc) * 2 + kk) * 64];
  };

  f32x4 acc[4][TJ2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 bb0[TJ2][2], bb1[TJ2][2];
#pragma unroll
  for (int t = 0; t < LEAD; ++t) stage_a(t);
  load_b2(bb0, 0);

  // K tile kt: load B(kt + 1), DMA A(kt + LEAD), wait until this wave's
  // A(kt) and B(kt) have landed (the VMEM ops issued after B(kt) - A(kt + 1),
  // B(kt + 1), A(kt + 2) - stay in flight), barrier (every wave's share of
  // A(kt) is in LDS), fragments, MFMAs. The compiler does not see the DMAs
  // (inline asm), so its own vmcnt before the first MFMA of a tile counts only
  // the B loads issued after B(kt): 2 TJ2, which also retires A(kt + 1), a
  // tile early.
  // WAR: A(kt + LEAD) overwrites slot (kt + LEAD) % NS, last read in
  // iteration kt + LEAD - NS <= kt - 2, which every wave finished before the
  // barrier of iteration kt - 1 (NS >= LEAD + 2).
  auto body = [&](int kt, const bf16x8(&bc)[TJ2][2], bf16x8(&bn)[TJ2][2]) {
    if (!(TAIL_ABL & 1)) load_b2(bn, kt + 1);
    if (!(TAIL_ABL & 2)) stage_a(kt + LEAD);
    static_assert(TJ2 == 4, "vmcnt below counts 1 + 2 * TJ2 + 1 = 10 ops");
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    if (!(TAIL_ABL & 4)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const uint8_t* as = ring + (kt % NS) * SLOT;
    bf16x8 fa[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[kk][i] = lds_read16(as + tail_swz(16 * i + fr, 4 * kk + fq));
    asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(fa[0][0]), "+v"(fa[0][1]), "+v"(fa[0][2]), "+v"(fa[0][3]));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j][0], fa[0][i], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fa[1][0]), "+v"(fa[1][1]), "+v"(fa[1][2]), "+v"(fa[1][3]));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TJ2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc[j][1], fa[1][i], acc[i][j], 0, 0, 0);
  };
  // fully unrolled (K1 is a template argument): with a runtime loop the
  // waitcnt pass merges the loop-carried B loads at the back edge and puts a
  // vmcnt(0) in front of every other tile's first MFMA (gfx950 ISA)
  static_assert(nkt % 2 == 0, "the two B buffers alternate");
#pragma unroll
  for (int kt = 0; kt < nkt; kt += 2) {
    body(kt, bb0, bb1);
    body(kt + 1, bb1, bb0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing ring stages land before LDS is reused

  // W3 fragments of this wave's columns, first half of K2, in flight during
  // the GEMM2 epilogue
  const bf16x8* w3w = W3p + int64_t(wid * TJ3) * NK2 * 2 * 64 + lane;
  bf16x8 wa[NK2 / 2][TJ3][2], wb[NK2 / 2][TJ3][2];
#pragma unroll
  for (int t = 0; t < NK2 / 2; ++t)
#pragma unroll
    for (int j = 0; j < TJ3; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wa[t][j][kk] = w3w[((j * NK2 + t) * 2 + kk) * 64];

  // GEMM2 epilogue: h2 = bf16(act2(acc + b2)) -> LDS, row m, column n at
  // 16-byte chunk (n / 8) ^ (m & 15) (conflict-free ds_read_b128 below)
  {
    const float lo = act2 == 1 ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < TJ2; ++j) {
      const int n = wid * (N2 / NW) + 16 * j + 4 * fq;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(b2 + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * i + fr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc[i][j][r] + b4[r], lo));
        *reinterpret_cast<bf16x4*>(h2s + m * H2P + (((n >> 3) ^ (m & 15)) << 4) + (n & 7) * 2) = o;
      }
    }
  }
  __syncthreads();
  if (TAIL_ABL & 8) {
    if (threadIdx.x < BM && m0 + int(threadIdx.x) < M) y[m0 + threadIdx.x] = bf2f(*reinterpret_cast<const bf16*>(h2s + threadIdx.x * H2P));
    return;
  }
#pragma unroll
  for (int t = 0; t < NK2 / 2; ++t)
#pragma unroll
    for (int j = 0; j < TJ3; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) wb[t][j][kk] = w3w[((j * NK2 + NK2 / 2 + t) * 2 + kk) * 64];

  // GEMM3: h3 = h2 W3^T over K2 = N2, A fragments from LDS
  f32x4 acc3[4][TJ3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ3; ++j) acc3[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto gemm3_tile = [&](int t, const bf16x8(&w)[TJ3][2]) {
    bf16x8 fa[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 16 * i + fr;
        fa[kk][i] = *reinterpret_cast<const bf16x8*>(h2s + m * H2P + (((8 * t + 4 * kk + fq) ^ fr) << 4));
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ3; ++j)
          acc3[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][kk], fa[kk][i], acc3[i][j], 0, 0, 0);
  };
#pragma unroll
  for (int t = 0; t < NK2 / 2; ++t) gemm3_tile(t, wa[t]);
#pragma unroll
  for (int t = 0; t < NK2 / 2; ++t) gemm3_tile(NK2 / 2 + t, wb[t]);

  // head: per-row partial dot over this wave's N3 / 8 columns, then the 4
  // lanes of a row (xor 16, 32), then the 8 waves through LDS
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  {
    const float lo = act3 == 1 ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < TJ3; ++j) {
      const int n = wid * (N3 / NW) + 16 * j + 4 * fq;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(b3 + n);
      const f32x4 h4 = *reinterpret_cast<const f32x4*>(hw + n);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[i] += fmaxf(acc3[i][j][r] + b4[r], lo) * h4[r];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = part[i];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (fq == 0) red[wid * BM + 16 * i + fr] = v;
  }
  __syncthreads();
  if (threadIdx.x < BM) {
    const int row = threadIdx.x;
    const int m = m0 + row;
    if (m < M) {
      float s = hbias;
      for (int e = 0; extra && e < extra_n; ++e) s += extra[e * extra_ld + m];
#pragma unroll
      for (int w = 0; w < NW; ++w) s += red[w * BM + row];
      y[m] = out_act == 2 ? sigmoidf(s) : s;
    }
  }
}

}  // namespace kern

hipError_t launch_mlp_tail(const void* X, int64_t ldx, int M, int K1, const void* W2p, const float* b2, int act2,
                           int N2, const void* W3p, const float* b3, int act3, int N3, const float* hw, float hbias,
                           const float* extra, int extra_n, int64_t extra_ld, int out_act, float* y, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (M < 0 || K1 != 1024 || N2 != 512 || N3 != 256 || extra_n < 0 ||
      (extra && extra_n > 1 && extra_ld < M))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((kern::mlp_tail_kernel<1024, 512, 256>), dim3((M + 63) / 64), dim3(512), 0, st,
                     static_cast<const kern::bf16*>(X), ldx, M, static_cast<const kern::bf16x8*>(W2p), b2, act2,
                     static_cast<const kern::bf16x8*>(W3p), b3, act3, hw, hbias, extra, extra_n, extra_ld, out_act, y);
  return hipGetLastError();
}

}  // namespace dtfs

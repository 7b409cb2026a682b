// K3b, one wave per SIMD (round 5): one DCN-v2 cross layer on the block-scaled
// MX-fp8 MFMA,
//   y = bf16(q W^T * sa[m] * sw[n] + b[n]),   z = bf16(x0 * y + xl)
// written as z (bf16) and / or per-column-tile partial head logits
// dot[tn, m] = z[m, 512 tn .. +512] . hw (the last layer only needs those).
// The same rounding as gemm.hip's cross_staged_epilogue (8-phase form).
//
// The structure of gather_gemm.hip without its gather: one 256-thread
// workgroup per CU, 128 rows x 512 columns, wave w owning columns 128 w ..
// +127 for all 128 rows (8 x 8 blocks of v_mfma_scale_f32_16x16x128_f8f6f4
// with unit block scales, the accumulator = the 256 AGPRs):
//   * W (e4m3) is the MFMA's A operand in fragment order (ops.pack_mx_frag:
//     lane (r, q) = (l & 15, l >> 4) of block (n16, k128) holds row 16 n16 + r,
//     K bytes [16 q, 16 q + 16) and [64 + 16 q, +16) - 1 KiB contiguous per
//     half), loaded by each wave straight into registers a K tile ahead;
//   * the activations q (e4m3 rows, 128 B per K tile) go through a 4-slot LDS
//     ring by LDS-DMA, three K tiles ahead;
//   * a K tile = 4 steps (two 16-column blocks each) of 16 MFMAs issued in
//     pairs; every load group goes out one op per MFMA pair in the step after
//     its registers' last read (WAR on in-flight MFMA sources, see
//     gather_gemm.hip), counted vmcnt / lgkmcnt waits, one barrier per tile;
//   * epilogue: y staged through LDS, then x0 / xl / z as whole 1 KiB row
//     segments.
//
// NOT part of the served build (rejected: 137-149 vs 122-125 us per layer at
// 16384 rows against the 8-phase form, profiles/r05_dcn_cross1w.md). Kept here
// for tools/native/cross1w_stamps.hip; build with -I csrc/kernels.
// hipcc-flags: -fno-slp-vectorize
#include "asm_io.h"
#include "common.h"
#include "launchers.h"

namespace dtfs {
bool cross1w_ok(int M, int N, int K);
int cross1w_tiles_n(int N);
hipError_t launch_cross1w(const CrossGemmArgs& args, const void* Wp, hipStream_t st);
}  // namespace dtfs

namespace dtfs {
namespace kern {

typedef int i32x8 __attribute__((ext_vector_type(8)));  // 32 x e4m3

namespace {
template <int N>
__device__ __forceinline__ void cwait_vm4(i32x4 (&x)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N));
}
template <int N>
__device__ __forceinline__ void cwait_lgkm2(i32x4& a, i32x4& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int OFF>
__device__ __forceinline__ i32x4 cread16(uint32_t addr) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
__device__ __forceinline__ i32x4 cgload16(const void* sbase, uint32_t voff) {
  i32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(v) : "v"(voff), "s"(sbase));
  return v;
}
__device__ __forceinline__ f32x4 mx16(const i32x4& alo, const i32x4& ahi, const i32x4& blo, const i32x4& bhi,
                                      const f32x4& c) {
  const i32x8 a = __builtin_shufflevector(alo, ahi, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8 b = __builtin_shufflevector(blo, bhi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}
}  // namespace

constexpr int kCx1wBM = 128, kCx1wBN = 512;

// Diagnostic build only (tools/native/cross1w_stamps.hip defines it): s_memtime
// stamps of one K tile in the middle of the loop (top, after steps 0, 1, 2, the
// barrier, step 3) plus entry / prologue / loop / epilogue, written by lane 0
// of each wave at the end.
#ifdef DTFS_CROSS1W_STAMPS
__device__ unsigned long long g_cross1w_stamps[4096][4][10];
__device__ unsigned long long g_cross1w_tiles[4096][4][32];  // top of every K tile (t < 32)
#define C1_TILE()                                                                       \
  do {                                                                                  \
    const unsigned long long c1_now = __builtin_amdgcn_s_memtime();                     \
    if (lane == 0 && blockIdx.x < 4096 && t < 32) g_cross1w_tiles[blockIdx.x][w][t] = c1_now; \
  } while (0)
#define C1_T(k)                                             \
  do {                                                      \
    if (t == c1_t) c1_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define C1_AT(k) c1_s[k] = __builtin_amdgcn_s_memtime()
#else
#define C1_T(k) \
  do {          \
  } while (0)
#define C1_AT(k) \
  do {           \
  } while (0)
#define C1_TILE() \
  do {            \
  } while (0)
#endif
// Ablations for the stamps tool only (wrong results): bit 0 drops the W
// loads, 1 the A DMAs, 2 the LDS fragment reads, 3 the per-tile barrier.
#ifndef CX_ABL
#define CX_ABL 0
#endif
// W touches (off): two cache-line touch loads per wave per K tile pulling the
// wave's W fragments of tile t+3 toward the L2 while tile t runs. Measured no
// gain (3871 vs 3801 cycles per K tile at 16384 rows, 187 vs 181 us).
#ifndef CX_TOUCH
#define CX_TOUCH 0
#endif

__global__ void __launch_bounds__(256, 1) cross1w_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                         const uint8_t* __restrict__ Wp, const float* __restrict__ bias,
                                                         const float* __restrict__ sa, const float* __restrict__ sw,
                                                         bf16* __restrict__ Z, int64_t ldz,
                                                         const bf16* __restrict__ X0, const bf16* __restrict__ XL,
                                                         int64_t ldx, const float* __restrict__ hw,
                                                         float* __restrict__ dot, int64_t ldd, int M, int N, int K) {
#ifdef DTFS_CROSS1W_STAMPS
  unsigned long long c1_s[10] = {};
  const int c1_t = K / 256;
#endif
  C1_AT(0);
  constexpr int BM = kCx1wBM, BN = kCx1wBN;
  constexpr int NS = 4;           // ring slots: tile t+1 (fragments), t+2 / t+3 (DMA in flight), t (free)
  constexpr int SLOT = BM * 128;  // 16 KiB
  constexpr int SP = BN * 2 + 16; // epilogue staging pitch (bytes)
  constexpr int SMEM = BM * SP > NS * SLOT ? BM * SP : NS * SLOT;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  const uint32_t ring = lds_addr(smem);

  const int KT = K / 128;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  // column-tile-major: an XCD's resident workgroups share one or two W column
  // panels (512 x K e4m3 = 1.4 MiB at K = 2816), which stay in its 4 MiB L2;
  // row-major order spread all of W (7.7 MiB) over every XCD and streamed it
  // from the MALL (1.69 vs ? PFLOP/s at 16384 x 2752 x 2816)
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = tile / tiles_m, tm = tile % tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int nblk = N / 16;  // valid 16-column blocks (N % 16 == 0)

  // ---- A ring: wave w DMAs rows 32 w + 8 k + (lane >> 3), k = 0..3, of every
  // K tile (lane i lands at +16 i = physical chunk lane & 7 of its row, which
  // holds logical chunk (lane & 7) ^ (row & 7))
  const int arow = 32 * w + (lane >> 3);
  const uint32_t a_chunk = uint32_t(((lane & 7) ^ ((lane >> 3) & 7)) << 4);
  const uint32_t ring_w = ring + 32 * w * 128;
  auto stage_a = [&](int u, int k) {  // 1 op
    const int uc = min(u, KT - 1);
    const int r = min(m0 + arow + 8 * k, M - 1);
    lds_dma16_s(A + int64_t(uc) * 128, uint32_t(int64_t(r) * lda) + a_chunk, ring_w + (u & (NS - 1)) * SLOT + k * 1024);
  };
  // ---- W fragments of wave w: column blocks jb = n0 / 16 + 8 w + j (clamped
  // to the last valid block on a ragged last tile), two 16-byte halves each
  i32x4 wf[8][2];
  const uint32_t w_lane = 16 * lane;
  auto load_w1 = [&](int u, int j, int h) {  // 1 op
    const int jb = min(n0 / 16 + 8 * w + j, nblk - 1);
    const uint8_t* frag = Wp + ((int64_t(jb) * KT + min(u, KT - 1)) * 2 + h) * 1024;
    wf[j][h] = cgload16(frag, w_lane);
  };
  // ---- x fragments: row 16 i + fr, chunks fq and fq + 4 (physical ^ (row & 7))
  i32x4 xf[8][2];
  const uint32_t xo_lo = fr * 128 + ((fq ^ (fr & 7)) << 4), xo_hi = fr * 128 + (((fq + 4) ^ (fr & 7)) << 4);
  // touch i (0, 1) of tile u: lane l -> fragment chunk l >> 2 (block j, half
  // h), cache lines 2 (l & 3) + i of its 8; into a dead LDS corner (the
  // epilogue's staging area, idle during the loop)
  const uint32_t touch_off = [&] {
    const int c = lane >> 2, jb = min(n0 / 16 + 8 * w + (c >> 1), nblk - 1);
    return uint32_t(((jb * KT) * 2 + (c & 1)) * 1024 + ((lane & 3) * 2) * 128);
  }();
  const uint32_t touch_lds = ring + NS * SLOT + 256 * w;
  auto touch_w = [&](int u, int i) {  // 1 op
    lds_dma4_s(Wp + int64_t(min(u, KT - 1)) * 2048 + 128 * i, touch_off, touch_lds);
  };
  auto read_x = [&](int u, int i) {  // 2 ops
    if (CX_ABL & 4) return;
    const uint32_t s = ring + (u & (NS - 1)) * SLOT + 2048 * i;
    xf[i][0] = cread16<0>(s + xo_lo);
    xf[i][1] = cread16<0>(s + xo_hi);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // step s runs column blocks 2 s and 2 s + 1; pair k: row block k of both
  auto pair = [&](int s, int k) {
    acc[k][2 * s] = mx16(wf[2 * s][0], wf[2 * s][1], xf[k][0], xf[k][1], acc[k][2 * s]);
    acc[k][2 * s + 1] = mx16(wf[2 * s + 1][0], wf[2 * s + 1][1], xf[k][0], xf[k][1], acc[k][2 * s + 1]);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // VMEM groups of tile t (one op per MFMA pair, in the step after the
  // registers' last read): G_s = W(t+1, column blocks 2 s, 2 s + 1) x 4, G0 / G1
  // + A(t+3, k = 0, 1 / 2, 3); G3(t-1) goes out in step 0 of tile t. The wait
  // for W(t, s) at the top of step s counts the ops issued after it: 12, 10,
  // 10, 12.
  // G2 also carries the two W touches of tile t+3 (CX_TOUCH): waits 14, 12, 12, 12.
  constexpr int TCH = CX_TOUCH ? 2 : 0;
  auto vm_op = [&](int t, int g, int i) {
    if (i < 4) {
      if (!(CX_ABL & 1)) load_w1(g == 3 ? t : t + 1, 2 * g + (i >> 1), i & 1);
    } else if (g == 2) {
      if (!(CX_ABL & 1)) touch_w(t + 3, i - 4);
    } else if (!(CX_ABL & 2)) {
      stage_a(t + 3, 2 * g + (i - 4));
    }
  };

  // ---- prologue: A(0), A(1); then G0(-1), G1(-1), G2(-1) (W(0, blocks 0-5),
  // A(2)); A(0)'s fragments 0-5 as step 3 leaves them
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(0, k);
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(1, k);
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int i = 0; i < (g == 2 ? 4 + TCH : 6); ++i) vm_op(-1, g, i);
  // A(0), A(1) landed (this wave's share)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 + TCH) : "memory");
  barrier();
#pragma unroll
  for (int i = 0; i < 6; ++i) read_x(0, i);
  C1_AT(1);

#pragma unroll 1
  for (int t = 0; t < KT; ++t) {
    C1_T(2);
    C1_TILE();
    // step 0 (column blocks 0, 1): fragments 6, 7 of A(t) read after pair 1
    cwait_vm4<12 + TCH>(*reinterpret_cast<i32x4(*)[4]>(&wf[0][0]));
    cwait_lgkm2<10>(xf[0][0], xf[0][1]);
    pair(0, 0);
    fence();
    cwait_lgkm2<8>(xf[1][0], xf[1][1]);
    pair(0, 1);
    vm_op(t, 3, 0);
    read_x(t, 6);
    read_x(t, 7);
    fence();
    cwait_lgkm2<10>(xf[2][0], xf[2][1]);
    pair(0, 2);
    vm_op(t, 3, 1);
    fence();
    cwait_lgkm2<8>(xf[3][0], xf[3][1]);
    pair(0, 3);
    vm_op(t, 3, 2);
    fence();
    cwait_lgkm2<6>(xf[4][0], xf[4][1]);
    pair(0, 4);
    vm_op(t, 3, 3);
    fence();
    cwait_lgkm2<4>(xf[5][0], xf[5][1]);
    pair(0, 5);
    fence();
    cwait_lgkm2<2>(xf[6][0], xf[6][1]);
    pair(0, 6);
    fence();
    cwait_lgkm2<0>(xf[7][0], xf[7][1]);
    pair(0, 7);
    fence();
    C1_T(3);
    // step 1 (blocks 2, 3): G0(t)
    cwait_vm4<10 + TCH>(*reinterpret_cast<i32x4(*)[4]>(&wf[2][0]));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(1, k);
      if (k >= 1 && k <= 6) vm_op(t, 0, k - 1);
      fence();
    }
    C1_T(4);
    // step 2 (blocks 4, 5): G1(t)
    cwait_vm4<10 + TCH>(*reinterpret_cast<i32x4(*)[4]>(&wf[4][0]));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(2, k);
      if (k >= 1 && k <= 6) vm_op(t, 1, k - 1);
      fence();
    }
    C1_T(5);
    // fragments of A(t) read (6 / 7 in step 0) and A(t+1) landed for every
    // wave (this step's wait retired G1(t-2)): one barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (!(CX_ABL & 8)) barrier();
    C1_T(6);
    // step 3 (blocks 6, 7): G2(t); fragments 0-5 of A(t+1), each two pairs
    // after its registers' last MFMA
    cwait_vm4<12>(*reinterpret_cast<i32x4(*)[4]>(&wf[6][0]));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= 2) read_x(t + 1, k - 2);
      pair(3, k);
      if (k >= 1 && k <= 4 + TCH) vm_op(t, 2, k - 1);
      fence();
    }
    C1_T(7);
  }
  C1_AT(8);
  // Retire the trailing prefetches before ANY epilogue instruction: the
  // compiler takes an asm load's output as written when the asm ends, so the
  // registers of the last (clamped, dead) prefetches are free to it after the
  // loop - without the sched_barrier it hoisted epilogue address math above the
  // wait into a W-fragment register still being loaded, a late return replaced
  // the address and the GPU faulted (memory aperture violation, graph replays
  // only). tests/test_kernel_resources.py runs tools/isa_hazards.py on this.
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();

  // ---- epilogue. Wave w owns rows w, w + 4, .. (32 of them), lane l the
  // tile's columns 8 l .. 8 l + 7. Its x0 / xl row segments are loaded 16 rows
  // at a time: row by row, every row waited out a whole memory round trip (the
  // epilogue took 43 k cycles, half the K loop's 84 k -
  // tools/native/cross1w_stamps.hip). (Loading the first batch before the y
  // staging spills at 512 registers.)
  int lane_e;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
  const int n = n0 + 8 * lane_e;
  const bool col_ok = n < N;  // N % 16 == 0: a lane's 8 columns exist together
  const int nr = min(n, N - 8);
  const bool same = XL == X0;
  // x0 / xl rows in batches of RB, two batches in registers: batch b + 1 is
  // loaded before batch b is computed and stored (vmcnt retires in order,
  // stores included: loads issued behind a batch's stores would wait for them)
  constexpr int RB = 8, NB = 32 / RB;
  bf16x8 xv[2][RB], lv[2][RB];
  auto load_rows = [&](int b) {
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int mc = min(m0 + w + 4 * (RB * b + i), M - 1);
      xv[b & 1][i] = *reinterpret_cast<const bf16x8*>(X0 + int64_t(mc) * ldx + nr);
    }
    if (!same) {
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int mc = min(m0 + w + 4 * (RB * b + i), M - 1);
        lv[b & 1][i] = *reinterpret_cast<const bf16x8*>(XL + int64_t(mc) * ldx + nr);
      }
    }
  };
  // y = bf16(acc * sa * sw + b) staged in LDS
  {
    float sam[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) sam[i] = sa[min(m0 + 16 * i + fr, M - 1)];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = 128 * w + 16 * j + 4 * fq;  // tile column of this lane's 4 values
      const int nc = min(n0 + c, N - 4);
      const f32x4 b4 = bias ? *reinterpret_cast<const f32x4*>(bias + nc) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(sw + nc);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(acc[i][j][r] * (s4[r] * sam[i]) + b4[r]);  // the 8-phase rounding
        *reinterpret_cast<bf16x4*>(smem + (16 * i + fr) * SP + c * 2) = o;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
  // ... then z = bf16(x0 * y + xl), written whole and / or dotted with hw
  {
    float w8[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) w8[e] = 0.f;
    if (hw && col_ok) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(hw + n);
      const f32x4 b = *reinterpret_cast<const f32x4*>(hw + n + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) w8[e] = a[e], w8[e + 4] = b[e];
    }
    load_rows(0);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b + 1 < NB) load_rows(b + 1);
      float d[RB];
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const int r = w + 4 * (RB * b + i);
        const int m = m0 + r;
        const bf16x8 y8 = *reinterpret_cast<const bf16x8*>(smem + r * SP + 16 * lane_e);
        const bf16x8 x8 = xv[b & 1][i];
        const bf16x8 l8 = same ? x8 : lv[b & 1][i];
        bf16x8 z8;
        d[i] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          z8[e] = f2bf(bf2f(x8[e]) * bf2f(y8[e]) + bf2f(l8[e]));
          d[i] += bf2f(z8[e]) * w8[e];
        }
        if (Z && col_ok && m < M) *reinterpret_cast<bf16x8*>(Z + int64_t(m) * ldz + n) = z8;
      }
      if (dot) {
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          float v = d[i];
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
          const int m = m0 + w + 4 * (RB * b + i);
          if (lane_e == 0 && m < M) dot[int64_t(tn) * ldd + m] = v;
        }
      }
    }
#ifdef DTFS_CROSS1W_STAMPS
    C1_AT(9);
    if (lane_e == 0 && blockIdx.x < 4096)
      for (int k = 0; k < 10; ++k) g_cross1w_stamps[blockIdx.x][w][k] = c1_s[k];
#endif
  }
}

}  // namespace kern

bool cross1w_ok(int M, int N, int K) { return M >= 1 && N >= 16 && N % 16 == 0 && K % 128 == 0 && K >= 128; }

int cross1w_tiles_n(int N) { return (N + kern::kCx1wBN - 1) / kern::kCx1wBN; }

hipError_t launch_cross1w(const CrossGemmArgs& a, const void* Wp, hipStream_t st) {
  if (a.M == 0) return hipSuccess;
  if (!cross1w_ok(a.M, a.N, a.K) || !a.A || !Wp || !a.sa || !a.sw || !a.X0 || !a.XL || (!a.Z && !a.dot) ||
      a.lda < a.K || a.ldx < a.N || (a.Z && a.ldz < a.N) || (a.dot && a.ldd < a.M) ||
      int64_t(a.M) * a.lda > (int64_t(1) << 32))
    return hipErrorInvalidValue;
  const int grid = ((a.M + kern::kCx1wBM - 1) / kern::kCx1wBM) * cross1w_tiles_n(a.N);
  hipLaunchKernelGGL(kern::cross1w_kernel, dim3(grid), dim3(256), 0, st, static_cast<const uint8_t*>(a.A), a.lda,
                     static_cast<const uint8_t*>(Wp), a.bias, a.sa, a.sw, static_cast<kern::bf16*>(a.Z), a.ldz,
                     static_cast<const kern::bf16*>(a.X0), static_cast<const kern::bf16*>(a.XL), a.ldx, a.hw, a.dot,
                     a.ldd, a.M, a.N, a.K);
  return hipGetLastError();
}

}  // namespace dtfs

// The whole DeepFM / Wide&Deep tower in ONE launch (round 6): K1 (weighted
// gather) + K2 (FM) + K4 x 3 (MLP 64F -> 1024 -> 512 -> 256) + K6 (head),
// after the resolve pass (rows_t / wts_t / first-order term, embed_resolve):
//
//   h1 = relu(sum_f bf16(w[m,f] T[row(m,f)]) . W1[:, 64f..64f+63]^T + b1)  bf16, LDS
//   h2 = act2(h1 W2^T + b2)                                                 bf16, LDS
//   h3 = act3(h2 W3^T + b3)                                                 fp32, registers
//   y[m] = sigmoid(h3[m] . hw + hbias + first-order(m) (+ FM(m)))
//
// Round 5 ran this as two kernels (gather_gemm.hip 128 x 512 tiles + mlp_tail.hip):
// 89 + 28 us per 16384-row step, h1 (32 MiB) written to HBM by the first and read
// back by the second (profiles/r05_deepfm_gg1w_kernels.md), and the tail streamed
// all of W2 into every 64-row workgroup anyway. Here one 256-thread workgroup per
// CU (16384 rows = 256 workgroups) owns 64 rows x ALL 1024 columns of h1 - the same
// 256 KiB of accumulators per CU (one wave per SIMD, 256 AGPRs each) - so h1 never
// leaves the CU:
//   * K loop (one K tile per field, as gather_gemm.hip): wave w owns h1 columns
//     256 w .. 256 w + 255 for all 64 rows, 8 x 2 blocks of
//     v_mfma_f32_32x32x16_bf16 (W1 = A operand in fragment order, ops.pack_frag32,
//     loaded straight into registers one K tile ahead; the gathered table rows =
//     B operand, LDS-DMA'd into a 4-slot ring three tiles ahead and weighted once
//     in LDS by a scale pass one tile ahead, which also accumulates the FM sums
//     of every row). Per K tile: 64 MFMAs per wave, 35 VMEM ops (32 W1
//     fragments, 2 table-row DMAs, 1 rows / weights DMA), one barrier;
//   * then h1 = relu(acc + b1) as bf16 into LDS (128 KiB, 16-byte chunks XOR
//     row-swizzled), GEMM2 (wave w: 128 of h2's 512 columns) with W2 fragments
//     from L2 one K tile ahead, h2 into LDS over h1, GEMM3 (64 columns per wave)
//     and the head reduced across lanes and waves in LDS; one score per row
//     straight to y (device or mapped pinned host memory).
// The price: every CU streams all of W1 per K tile (128 KiB instead of 64 KiB);
// W1 (5.6 MB) stays L2 / Infinity-Cache resident across the 256 workgroups.
//
// Hazard rules of gather_gemm.hip apply unchanged (every hot-loop memory op is
// inline asm with counted waits; a load overwrites an MFMA operand only whole
// MFMA pairs after its last read; the registers of the dead trailing
// prefetches are free only after the post-loop wait, pinned by sched_barrier).
// hipcc-flags: -fno-slp-vectorize
// MFMA: D = W_frag x X_frag^T: lane (r, h) = (l & 31, l >> 5) holds
// C[m = 32 im + r][n = 32 jn + (g & 3) + 8 (g >> 2) + 4 h] in register g.
#include <utility>

#include "asm_io.h"
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Diagnostic build only (tools/native/gm_stamps.hip defines it): s_memtime
// stamps - entry, prologue end, the six step boundaries of one K tile in the
// middle of the loop, loop end, h1 stored, GEMM2 done, h2 stored, head done -
// written by lane 0 of each wave at the end.
#ifdef DTFS_GM_STAMPS
__device__ unsigned long long g_gm_stamps[1024][4][16];
#define GM_T(k)                                             \
  do {                                                      \
    if (t == gm_t) gm_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define GM_AT(k)                              \
  do {                                        \
    gm_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define GM_T(k) \
  do {          \
  } while (0)
#define GM_AT(k) \
  do {           \
  } while (0)
#endif

namespace {
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read16_at(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ i32x4 ds_read16i_at(uint32_t addr) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ int ds_read4_at(uint32_t addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ void ds_write16_at(uint32_t addr, const i32x4& v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_lgkm2(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_vm8(bf16x8 (&x)[4], bf16x8 (&y)[4]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3])
               : "n"(N));
}
}  // namespace

// The h1 / h2 tiles in LDS: row m at m * pitch, 16-byte chunk c at c ^ (m & 15)
// (a 16-lane ds_read_b128 group reads 16 rows of one logical chunk: 16 banks groups)
__device__ __forceinline__ uint32_t hswz(int m, int c, int pitch) { return m * pitch + ((c ^ (m & 15)) << 4); }

template <int N>
__device__ __forceinline__ void wait_vm_4(bf16x8& a, bf16x8& b, bf16x8& c, bf16x8& d) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_vm_2(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <class Fn, int... I>
__device__ __forceinline__ void gm_sfor_(Fn&& fn, std::integer_sequence<int, I...>) {
  (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void gm_sfor(Fn&& fn) {
  gm_sfor_(fn, std::make_integer_sequence<int, N>{});
}

// One of the tail GEMMs on a tile already in LDS: acc[jn][im] += W_frag(jn) x
// H_frag(im)^T over NK K tiles of 64, H = the 64-row bf16 activation at LDS
// byte address hbase with row pitch PITCH (chunk c of row m at c ^ (m & 15)),
// W = this wave's NJ packed 32-column blocks (ops.pack_frag32, [NJ][NK][4][64]
// fragments from Wb). Every load is inline asm with a counted wait (left to
// the compiler, these loads sank to their MFMAs: one exposed L2 round trip per
// MFMA pair, 99 k cycles for GEMM2); K step s of tile kt refills the two
// buffers' registers that K step s of tile kt - 1 read (a whole tile ago).
template <int NJ, int NK, int PITCH>
__device__ __forceinline__ void tail_gemm(const bf16x8* __restrict__ Wb, uint32_t hbase, int r32, int h,
                                          f32x16 (&acc)[NJ][2]) {
  static_assert(PITCH % 256 == 0 && NK % 2 == 0, "tail_gemm shape");
  // lane's row 32 im + r32, chunk 8 kt + 2 s + h at ((h ^ (r32 & 15)) ^ (2 s + 8 (kt & 1))) + 16 (kt >> 1)
  const uint32_t hb0 = r32 * PITCH + ((h ^ (r32 & 15)) << 4);  // relative: the XOR touches bits 4-7 only
  const uint32_t hb1 = hb0 + 32 * PITCH;
  const uint32_t voff = 16 * (r32 + 32 * h);
  bf16x8 wf[2][NJ][4], hf[2][2][4];
  auto issue = [&](auto KT, auto S) {
    constexpr int kt = decltype(KT)::value, s = decltype(S)::value;
#pragma unroll
    for (int jn = 0; jn < NJ; ++jn) wf[kt & 1][jn][s] = gload16_s(Wb + ((jn * NK + kt) * 4 + s) * 64, voff);
    constexpr uint32_t x = uint32_t(2 * s + 8 * (kt & 1)) << 4;
    constexpr int off = (kt >> 1) * 256;
    hf[kt & 1][0][s] = ds_read16_at<off>(hbase + (hb0 ^ x));
    hf[kt & 1][1][s] = ds_read16_at<off>(hbase + (hb1 ^ x));
  };
  gm_sfor<4>([&](auto S) { issue(std::integral_constant<int, 0>{}, S); });
  gm_sfor<NK>([&](auto KT) {
    constexpr int kt = decltype(KT)::value, b = kt & 1;
    gm_sfor<4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      constexpr bool more = kt + 1 < NK;
      constexpr int nv = NJ * (3 - s) + (more ? NJ * s : 0);
      constexpr int nl = 2 * (3 - s) + (more ? 2 * s : 0);
      if constexpr (NJ == 4)
        wait_vm_4<nv>(wf[b][0][s], wf[b][1][s], wf[b][2][s], wf[b][3][s]);
      else
        wait_vm_2<nv>(wf[b][0][s], wf[b][1][s]);
      wait_lgkm2<nl>(hf[b][0][s], hf[b][1][s]);
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn)
#pragma unroll
        for (int im = 0; im < 2; ++im)
          acc[jn][im] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[b][jn][s], hf[b][im][s], acc[jn][im], 0, 0, 0);
      if constexpr (more) issue(std::integral_constant<int, kt + 1>{}, S);
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

template <bool FM>
__global__ void __launch_bounds__(256, 1)
    gather_mlp_kernel(EmbedArgs ea, uint64_t magic, int F, const bf16x8* __restrict__ W1p,
                      const float* __restrict__ b1, const bf16x8* __restrict__ W2p, const float* __restrict__ b2,
                      int act2, const bf16x8* __restrict__ W3p, const float* __restrict__ b3, int act3,
                      const float* __restrict__ hw, float hbias, int M, int out_act, float* __restrict__ y) {
  constexpr int BM = 64;
  constexpr int N1 = 1024, N2 = 512, N3 = 256;
  constexpr int NS = 4;   // A ring slots: tile t+1 (scale pass, then fragments), t+2 / t+3 (DMA), t (free)
  constexpr int SLOT = BM * 128;
  constexpr int FMAX = 64;
  constexpr int TROWS = NS * SLOT, TWTS = TROWS + FMAX * BM * 4;  // resolved rows / weights [F][64], field-major
  constexpr int H1P = N1 * 2, H2P = N2 * 2;
  constexpr int HOFF = BM * H1P;  // head partials [4][64] fp32, the FM terms [64], the first-order terms [64]
  constexpr int BOFF = HOFF + 4 * BM * 4 + 2 * BM * 4;  // b1 | b2 | b3 | hw, fp32, staged once
  constexpr int SMEM = BOFF + (N1 + N2 + N3 + N3) * 4;
  static_assert(TWTS + FMAX * BM * 4 <= HOFF, "the K loop's ring and row tables live inside the h1 tile");
  const uint8_t* const table = static_cast<const uint8_t*>(ea.table);
  const int Vm1 = int(ea.V - 1);
#ifdef DTFS_GM_STAMPS
  unsigned long long gm_s[16] = {};
  const int gm_t = F / 2;
#endif
  GM_AT(0);
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  int32_t* const rows_l = reinterpret_cast<int32_t*>(smem + TROWS);
  float* const wts_l = reinterpret_cast<float*>(smem + TWTS);
  float* const red = reinterpret_cast<float*>(smem + HOFF);
  float* const fmv = red + 4 * BM;
  float* const firstv = fmv + BM;
  float* const b1s = reinterpret_cast<float*>(smem + BOFF);
  float* const b2s = b1s + N1;
  float* const b3s = b2s + N2;
  float* const hws = b3s + N3;
  const uint32_t aring_lds = lds_addr(smem);
  const uint32_t rows_lds = lds_addr(rows_l), wts_lds = lds_addr(wts_l);

  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int T = threadIdx.x;
  const int lane = T & 63;
  const int w = __builtin_amdgcn_readfirstlane(T >> 6);
  const int r32 = lane & 31, h = lane >> 5;

  // ---- staging (VMEM: every wave issues the same number per tile)
  // A tile u: wave w DMAs rows R = 16 w + 8 k + (lane >> 3), k = 0..1 (1 KiB
  // each); lane i lands at +16 i = physical chunk lane & 7 of row R, which
  // holds logical chunk (lane & 7) ^ (R & 7)
  const int arow0 = 16 * w + (lane >> 3);
  const int a_src = ((lane & 7) ^ ((lane >> 3) & 7)) << 4;
  const uint32_t aring_w = aring_lds + 16 * w * 128;
  const uint32_t idx_off = 4 * arow0;
  int aidx[2];
  auto read_idx = [&](int u) {  // 2 LDS ops (tiles past the last re-read it: branch-free loop)
    const uint32_t base = rows_lds + min(u, F - 1) * (BM * 4) + idx_off;
    aidx[0] = ds_read4_at<0>(base);
    aidx[1] = ds_read4_at<32>(base);
  };
  auto stage_a = [&](int u, int k) {  // 1 op; aidx of tile u landed (table < 4 GiB: a 32-bit offset)
    const int rr = min(max(aidx[k], 0), Vm1);
    lds_dma16_s(table, uint32_t(rr) * 128u + a_src, aring_w + (u & (NS - 1)) * SLOT + k * 1024);
  };
  // W1 fragments of wave w: packed blocks 8 w + jn, layout [N1/32][F][4][64][8]
  const bf16x8* wpw = W1p + int64_t(8 * w) * F * 4 * 64;
  const uint32_t w_lane = 16 * lane;
  bf16x8 wf[8][4];
  auto load_w1 = [&](int u, int jn, int s) {  // 1 op
    wf[jn][s] = gload16_s(wpw + ((int64_t(jn) * F + min(u, F - 1)) * 4 + s) * 64, w_lane);
  };

  // ---- x fragments (the MFMA's B operand): row 32 im + r32, K 16 s + 8 h .. +7
  // = logical chunk 2 s + h at physical (2 s + h) ^ (r32 & 7); bits 5-6 of the
  // byte offset are s ^ ((r32 >> 1) & 3), so K step s XORs (s << 5) into one base
  bf16x8 xf[2][4];
  const uint32_t xo0 = r32 * 128 + ((h ^ (r32 & 1)) << 4) + (((r32 >> 1) & 3) << 5);
  auto read_xs = [&](int u, int s) {  // 2 ops: K step s of both row blocks
    const uint32_t a = aring_lds + (u & (NS - 1)) * SLOT + (xo0 ^ uint32_t(s << 5));
    xf[0][s] = ds_read16_at<0>(a);
    xf[1][s] = ds_read16_at<4096>(a);
  };
  // ---- scale pass: thread T rescales logical chunk T & 7 of rows (T >> 3) +
  // 32 q, q = 0, 1, and (DeepFM) accumulates both rows' FM sums
  const int sc_c = T & 7, sc_r0 = T >> 3;
  const uint32_t sc_off = sc_r0 * 128 + ((sc_c ^ (sc_r0 & 7)) << 4);
  i32x4 sv[2];
  int swt[2];
  float fs[2][8], fsq[2] = {0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int d = 0; d < 8; ++d) fs[a][d] = 0.f;
  auto scale_read = [&](int u) {  // 4 ops
    const uint32_t base = aring_lds + (u & (NS - 1)) * SLOT + sc_off;
    const uint32_t wb = wts_lds + min(u, F - 1) * (BM * 4) + 4 * sc_r0;
    sv[0] = ds_read16i_at<0>(base);
    swt[0] = ds_read4_at<0>(wb);
    sv[1] = ds_read16i_at<4096>(base);
    swt[1] = ds_read4_at<128>(wb);
  };
  auto scale_wait = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(sv[0]), "+v"(sv[1]), "+v"(swt[0]), "+v"(swt[1]));
  };
  i32x4 so[2];
  auto scale_pair = [&](int u, int q, int p) {
    // u == F: the trailing re-staged tile (never multiplied): zero weight, so
    // the FM sums stay exact without a branch
    const float wt = u < F ? __int_as_float(swt[q]) : 0.f;
    const float a = __uint_as_float(uint32_t(sv[q][p]) << 16) * wt;
    const float b = __uint_as_float(uint32_t(sv[q][p]) & 0xffff0000u) * wt;
    so[q][p] = __builtin_bit_cast(int, __builtin_convertvector((f32x2){a, b}, bf16x2));
    if constexpr (FM) {
      fs[q][2 * p] += a;
      fs[q][2 * p + 1] += b;
      fsq[q] += a * a;
      fsq[q] += b * b;
    }
    if (p == 3) ds_write16_at<0>(aring_lds + (u & (NS - 1)) * SLOT + sc_off + 4096 * q, so[q]);
  };

  f32x16 acc[8][2];  // [jn][im]
#pragma unroll
  for (int jn = 0; jn < 8; ++jn)
#pragma unroll
    for (int im = 0; im < 2; ++im)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[jn][im][g] = 0.f;
  auto mfma1 = [&](int jn, int im, int s) {
    acc[jn][im] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[jn][s], xf[im][s], acc[jn][im], 0, 0, 0);
  };
  // pair k of step st: K step s = k >> 1 of column block 2 st + (k & 1), both row blocks
  auto pair = [&](int st, int k) {
    mfma1(2 * st + (k & 1), 0, k >> 1);
    mfma1(2 * st + (k & 1), 1, k >> 1);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto wait_idx = [&] { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aidx[0]), "+v"(aidx[1])::"memory"); };
#define WAIT_XS(N, s) wait_lgkm2<N>(xf[0][s], xf[1][s])

  // ---- VMEM per tile t, one op after each MFMA pair of the step after the
  // one that last read the registers it refills (op i of a W group refills
  // wf[jn = 2 g' + (i & 1)][s = i >> 1], last read by pair i of its step):
  //   step 0: W(t, 6..7) x 8
  //   step 1: W(t+1, 0..1) x 8, A(t+3, 0)
  //   step 2: W(t+1, 2..3) x 8, A(t+3, 1)
  //   step 3: W(t+1, 4..5) x 8
  // so the counted wait for W(t, 2 st .. 2 st + 1) at the top of step st is
  // vmcnt 18, 17, 17, 18 (the ops issued after it, in order). vmcnt retires in
  // issue order: step 2's wait retires A(t+2) (issued at tile t-1) before the
  // tile's barrier. The rows / weights of every tile are resolved into LDS by
  // the prologue (no rows ring).
  auto vm_op = [&](int t, int g, int i) {
    if (g == 3) {
      load_w1(t, 6 + (i & 1), i >> 1);
    } else if (i < 8) {
      load_w1(t + 1, 2 * g + (i & 1), i >> 1);
    } else {
      stage_a(t + 3, g);
    }
  };

  // the epilogues' biases and head weights, once into LDS (outside the rings;
  // retired by the prologue's waits before the loop counts anything)
  reinterpret_cast<f32x4*>(b1s)[T] = reinterpret_cast<const f32x4*>(b1)[T];
  if (T < N2 / 4) reinterpret_cast<f32x4*>(b2s)[T] = reinterpret_cast<const f32x4*>(b2)[T];
  if (T < N3 / 4) {
    reinterpret_cast<f32x4*>(b3s)[T] = reinterpret_cast<const f32x4*>(b3)[T];
    reinterpret_cast<f32x4*>(hws)[T] = reinterpret_cast<const f32x4*>(hw)[T];
  }
  // W1 fragments of tile 0 for steps 0-2 (the groups of "tile -1" in the
  // loop's issue order): 24 loads whose latency hides behind the resolve
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int i = 0; i < 8; ++i) vm_op(-1, g, i);
  // ---- resolve (K0 + the gather's front half, in the kernel: no resolve pass,
  // no kernel boundary): this workgroup's 64 rows x F fields -> clamped table
  // rows and weights, field-major in LDS, plus each row's first-order term
  // bias + sum_f lin[row] w. Thread T: row T & 63, fields T >> 6, +4, +8, ...;
  // every id / weight load of a thread goes out before the first use, then
  // every lin load: two dependent round trips after the row descriptor.
  {
    constexpr int KR = FMAX / 4;
    const int rr = T & 63, f0 = T >> 6;
    const int b = m0 + rr;
    ArenaRow ar{nullptr, nullptr, false, kArenaAllWeights, 4};
    if (ea.arena && b < ea.B) ar = arena_row(static_cast<const uint8_t*>(ea.arena), kArenaPayloadOff, b);
    int64_t id[KR];
    float wv[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int f = f0 + 4 * k;
      id[k] = 0;
      wv[k] = 0.f;
      if (f < F && b < ea.B) {
        if (ea.arena) {
          if (ar.ids) arena_feature(ar, f, id[k], wv[k]);
        } else {
          id[k] = ea.ids64 ? static_cast<const int64_t*>(ea.ids)[int64_t(b) * ea.ids_ld + f]
                           : int64_t(static_cast<const int32_t*>(ea.ids)[int64_t(b) * ea.ids_ld + f]);
          wv[k] = !ea.wts ? 1.f
                  : ea.wts16 ? __uint_as_float(uint32_t(static_cast<const uint16_t*>(ea.wts)[int64_t(b) * ea.wts_ld + f]) << 16)
                             : static_cast<const float*>(ea.wts)[int64_t(b) * ea.wts_ld + f];
        }
      }
    }
    float lsum = 0.f;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int f = f0 + 4 * k;
      if (f < F) {
        int64_t g = magic ? hash_row_magic(id[k], ea.modulo, magic) : hash_row(id[k], ea.modulo);
        g = g < 0 ? 0 : (g > Vm1 ? Vm1 : g);  // memory safety whatever the ids say
        rows_l[f * BM + rr] = int32_t(g);
        wts_l[f * BM + rr] = wv[k];
        if (ea.lin) lsum += ea.lin[g] * wv[k];
      }
    }
    red[f0 * BM + rr] = lsum;
  }
  __syncthreads();
  if (T < BM) firstv[T] = ea.bias + red[T] + red[BM + T] + red[2 * BM + T] + red[3 * BM + T];
  // ---- prologue: A(0), A(1), A(2); A(0) scaled; idx(3) read; K steps 0-2 of
  // A(0)'s fragments in flight as step 3 of a tile leaves them. Tile 0's
  // counted waits hold: every W load of "tile -1" is retired below, and only
  // A(2) stays in flight into the loop (fewer ops than the waits allow)
  read_idx(0);
  wait_idx();
  stage_a(0, 0);
  stage_a(0, 1);
  read_idx(1);
  wait_idx();
  stage_a(1, 0);
  stage_a(1, 1);
  read_idx(2);
  wait_idx();
  stage_a(2, 0);
  stage_a(2, 1);
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // A(0), A(1) landed (this wave's share); A(2) in flight
  barrier();
  scale_read(0);
  scale_wait();
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) scale_pair(0, q, p);
  read_idx(3);
  wait_idx();
  barrier();
  read_xs(0, 0);
  read_xs(0, 1);
  read_xs(0, 2);
  GM_AT(1);

  // ---- main loop: K tile t = field t, 4 steps of 8 MFMA pairs
#pragma unroll 1
  for (int t = 0; t < F; ++t) {
    if constexpr (FM) {
      // the FM sums are complete once tile F-1 is scaled (during tile F-2):
      // the last tile parks each row's term in LDS (outside the rings)
      if (t == F - 1) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          float part = -fsq[a];
#pragma unroll
          for (int d = 0; d < 8; ++d) part += fs[a][d] * fs[a][d];
          part += __shfl_xor(part, 1, 64);
          part += __shfl_xor(part, 2, 64);
          part += __shfl_xor(part, 4, 64);
          if (sc_c == 0) fmv[sc_r0 + 32 * a] = 0.5f * part;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the shuffles / store, not mid-step 0
      }
    }
    // step 0: A(t)'s fragments land K step by K step; W(t, 6..7), ring(t+5)
    wait_vm8<18>(wf[0], wf[1]);
    GM_T(2);
    WAIT_XS(4, 0);
    pair(0, 0);
    vm_op(t, 3, 0);
    fence();
    pair(0, 1);
    vm_op(t, 3, 1);
    fence();
    read_xs(t, 3);  // registers last read by pairs 6-7 of step 3, tile t-1
    WAIT_XS(4, 1);
    pair(0, 2);
    vm_op(t, 3, 2);
    fence();
    pair(0, 3);
    vm_op(t, 3, 3);
    fence();
    WAIT_XS(2, 2);
    pair(0, 4);
    vm_op(t, 3, 4);
    fence();
    pair(0, 5);
    vm_op(t, 3, 5);
    fence();
    WAIT_XS(0, 3);
    scale_read(t + 1);
    pair(0, 6);
    vm_op(t, 3, 6);
    fence();
    pair(0, 7);
    vm_op(t, 3, 7);
    fence();
    GM_T(3);
    // step 1: the scale pass's chunk of rows r (q = 0); W(t+1, 0..1), A(t+3, 0)
    wait_vm8<17>(wf[2], wf[3]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(1, k);
      if (k == 0) scale_wait();  // the scale reads had step 0's last two pairs + this one
      if (!(k & 1)) scale_pair(t + 1, 0, k >> 1);
      vm_op(t, 0, k);
      if (k == 7) vm_op(t, 0, 8);
      fence();
    }
    GM_T(4);
    // step 2: rows r + 32 (q = 1); W(t+1, 2..3), A(t+3, 1); then the rows of A(t+4)
    wait_vm8<17>(wf[4], wf[5]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(2, k);
      if (!(k & 1)) scale_pair(t + 1, 1, k >> 1);
      vm_op(t, 1, k);
      if (k == 7) {
        vm_op(t, 1, 8);
        read_idx(t + 4);
      }
      fence();
    }
    GM_T(5);
    wait_idx();  // + this wave's scale writes
    barrier();
    GM_T(6);
    // step 3: K steps 0-2 of A(t+1) stream in, each two pairs after its
    // registers' last use; W(t+1, 4..5)
    wait_vm8<18>(wf[6], wf[7]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k == 4) read_xs(t + 1, 0);
      if (k == 6) read_xs(t + 1, 1);
      pair(3, k);
      vm_op(t, 2, k);
      fence();
    }
    read_xs(t + 1, 2);
    GM_T(7);
  }
#undef WAIT_XS
  // the trailing (re-staged, unread) loads land before the LDS is reused
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  GM_AT(8);
  // lane-derived indices of everything below are recomputed from a volatile
  // read of the lane id (kept live across the loop they spilled to scratch in
  // gather_gemm.hip; scratch-free is a test)
  int lane_e;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
  const int r32e = lane_e & 31, he = lane_e >> 5;
  int tid_e;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid_e) : "v"(lane_e));
  tid_e += 64 * w;
  __syncthreads();

  // ---- h1 = relu(acc + b1) -> bf16 -> LDS (row m, column n: chunk n / 8 of
  // row m); the biases come from the LDS copy the prologue made
#pragma unroll
  for (int jn = 0; jn < 8; ++jn) {
    f32x4 b4[4];
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) b4[g4] = *reinterpret_cast<const f32x4*>(b1s + 256 * w + 32 * jn + 8 * g4 + 4 * he);
#pragma unroll
    for (int im = 0; im < 2; ++im) {
      const f32x16 av = acc[jn][im];
      const int m = 32 * im + r32e;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = 256 * w + 32 * jn + 8 * g4;  // + 4 he: the second half of chunk n / 8
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(av[4 * g4 + e] + b4[g4][e], 0.f));
        *reinterpret_cast<bf16x4*>(smem + hswz(m, n >> 3, H1P) + 8 * he) = o;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __syncthreads();
  GM_AT(9);

  // ---- GEMM2: wave w computes h2 columns 128 w .. 128 w + 127 of all 64 rows
  // (K = 1024), explicit two-buffer pipeline (tail_gemm)
  {
    f32x16 acc2[4][2];
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
#pragma unroll
      for (int im = 0; im < 2; ++im)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc2[jn][im][g] = 0.f;
    tail_gemm<4, N1 / 64, H1P>(W2p + int64_t(4 * w) * (N1 / 64) * 4 * 64, aring_lds, r32e, he, acc2);
    GM_AT(10);
    __syncthreads();  // every wave is done reading h1: h2 goes over it
    const float lo2 = act2 == 1 ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      f32x4 b4[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        b4[g4] = *reinterpret_cast<const f32x4*>(b2s + 128 * w + 32 * jn + 8 * g4 + 4 * he);
#pragma unroll
      for (int im = 0; im < 2; ++im) {
        const int m = 32 * im + r32e;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int n = 128 * w + 32 * jn + 8 * g4;
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(acc2[jn][im][4 * g4 + e] + b4[g4][e], lo2));
          *reinterpret_cast<bf16x4*>(smem + hswz(m, n >> 3, H2P) + 8 * he) = o;
        }
      }
    }
  }
  __syncthreads();
  GM_AT(11);

  // ---- GEMM3: wave w computes h3 columns 64 w .. 64 w + 63 (K = 512), then
  // the head: h3 . hw per row over lanes, then over waves in LDS
  {
    f32x16 acc3[2][2];
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int im = 0; im < 2; ++im)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc3[jn][im][g] = 0.f;
    tail_gemm<2, N2 / 64, H2P>(W3p + int64_t(2 * w) * (N2 / 64) * 4 * 64, aring_lds, r32e, he, acc3);
    const float lo3 = act3 == 1 ? 0.f : -__builtin_huge_valf();
    float part[2] = {0.f, 0.f};
#pragma unroll
    for (int jn = 0; jn < 2; ++jn)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = 64 * w + 32 * jn + 8 * g4 + 4 * he;
        const f32x4 bb = *reinterpret_cast<const f32x4*>(b3s + n);
        const f32x4 hh = *reinterpret_cast<const f32x4*>(hws + n);
#pragma unroll
        for (int im = 0; im < 2; ++im)
#pragma unroll
          for (int e = 0; e < 4; ++e) part[im] += fmaxf(acc3[jn][im][4 * g4 + e] + bb[e], lo3) * hh[e];
      }
#pragma unroll
    for (int im = 0; im < 2; ++im) {
      const float v = part[im] + __shfl_xor(part[im], 32, 64);
      if (he == 0) red[w * BM + 32 * im + r32e] = v;
    }
  }
  __syncthreads();
  if (tid_e < BM) {
    const int m = m0 + tid_e;
    if (m < M) {
      float s = hbias + firstv[tid_e];
      if constexpr (FM) s += fmv[tid_e];
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) s += red[ww * BM + tid_e];
      y[m] = out_act == 2 ? sigmoidf(s) : s;
    }
  }
#ifdef DTFS_GM_STAMPS
  GM_AT(12);
  if (lane_e == 0 && blockIdx.x < 1024)
    for (int k = 0; k < 13; ++k) g_gm_stamps[blockIdx.x][w][k] = gm_s[k];
#endif
}

}  // namespace kern

bool gather_mlp_ok(int64_t Mp, int N1, int K1, int N2, int N3, int F, int64_t V) {
  return N1 == 1024 && N2 == 512 && N3 == 256 && K1 == 64 * F && Mp % 64 == 0 && F >= 1 && F <= 64 && V >= 1 &&
         V <= (int64_t(1) << 25);
}

hipError_t launch_gather_mlp(const EmbedArgs& a, const void* W1p, const float* b1, const void* W2p, const float* b2,
                             int act2, const void* W3p, const float* b3, int act3, const float* hw, float hbias,
                             bool fm, int out_act, float* y, hipStream_t st) {
  if (a.B == 0) return hipSuccess;
  const int64_t Mp = (int64_t(a.B) + 63) / 64 * 64;
  if (!gather_mlp_ok(Mp, 1024, 64 * a.F, 512, 256, a.F, a.V) || a.B < 0 || a.modulo <= 0 || !a.table ||
      (!a.arena && !a.ids) || a.modulo_f || a.shard_lo_f || !W1p || !b1 || !W2p || !b2 || !W3p || !b3 || !hw || !y)
    return hipErrorInvalidValue;
  const uint64_t magic = a.modulo < (int64_t(1) << 32) ? ~uint64_t(0) / uint64_t(a.modulo) : 0;
  const int grid = int(Mp / 64);
  if (fm)
    hipLaunchKernelGGL((kern::gather_mlp_kernel<true>), dim3(grid), dim3(256), 0, st, a, magic, a.F,
                       static_cast<const kern::bf16x8*>(W1p), b1, static_cast<const kern::bf16x8*>(W2p), b2, act2,
                       static_cast<const kern::bf16x8*>(W3p), b3, act3, hw, hbias, a.B, out_act, y);
  else
    hipLaunchKernelGGL((kern::gather_mlp_kernel<false>), dim3(grid), dim3(256), 0, st, a, magic, a.F,
                       static_cast<const kern::bf16x8*>(W1p), b1, static_cast<const kern::bf16x8*>(W2p), b2, act2,
                       static_cast<const kern::bf16x8*>(W3p), b3, act3, hw, hbias, a.B, out_act, y);
  return hipGetLastError();
}

}  // namespace dtfs

// K1 fused into K4, one wave per SIMD (round 5): the DeepFM / Wide&Deep first
// MLP layer straight from the embedding table,
//   C[m, n] = act( sum_f bf16(w[m,f] * T[row(m,f)]) . W[n, 64f .. 64f+63] + b[n] )
// plus (DeepFM) the second-order FM term of every row, on the same inputs as
// gemm.hip's gemm_gather_kernel (rows_t / wts_t from embed_resolve_kernel).
//
// Why a second form: the 8-phase gemm_gather_kernel (2 waves per SIMD, 256x256
// tiles, both operands LDS-DMA'd) measured ~4500 cycles per K tile against the
// ~2050 its MFMAs need (profiles/r04_gg_stamps.md): every inter-barrier
// interval is max(one group's MFMAs, the other group's LDS reads + 4-9 DMA
// issues), and the random-row DMAs + the B tile's DMAs + 24 fragment reads per
// wave and tile outran the 16 MFMAs they were paired with. Here:
//   * one 256-thread workgroup per CU, ONE wave per SIMD (512 registers each):
//     a 128-row x 512-column tile, wave w owns columns 128 w .. 128 w + 127 for
//     all 128 rows: 4 x 4 blocks of v_mfma_f32_32x32x16_bf16 (acc = the 256
//     AGPRs). 32x32x16 rather than 16x16x32: each MFMA holds vector issue for 8
//     of its 32 cycles (8 of 16), so a K tile's 64 MFMAs leave 1536 issue
//     cycles for the scale pass, the loads and the address math, against 1024
//     for the 128 16x16x32 MFMAs of the same work (measured: 3900 vs 3800
//     cycles per K tile with the 16x16 form's 60 % more instructions);
//   * W never touches LDS: it is the MFMA's A operand, kept in 32x32x16
//     fragment order (ops.pack_frag32), and each wave loads its own fragments
//     straight into registers one K tile ahead, rolling: W(t+1, jn) refills the
//     registers of W(t, jn) right after step jn's MFMAs (4 steps per tile, one
//     per 32-column block jn);
//   * A (the gathered table rows, 128 x 128 B per field) goes through a 4-slot
//     LDS ring by LDS-DMA, three K tiles ahead of its MFMAs; the weights are
//     applied ONCE per element in LDS by a scale pass over tile t+1 while tile
//     t's MFMAs run (the unfused gather's bf16(w * e) rounding, bit for bit),
//     which also accumulates the FM sums; A fragments (the MFMA's B operand)
//     of tile t+1 are read into registers during the last step of tile t;
//   * one barrier per K tile; every vmcnt / lgkmcnt is counted (all hot-loop
//     memory operations are inline asm, csrc/kernels/asm_io.h);
//   * WAR on MFMA sources: a load may overwrite an MFMA's operand registers
//     only a whole MFMA group (4 MFMAs, 128 cycles) after the MFMA issued - an
//     in-flight 32x32x16 still reads them, the inline-asm loads get no hazard
//     padding from the compiler, and a ds_read can land within that window
//     (measured: half the outputs wrong at 43 fields with the prefetch right
//     behind the MFMAs). sched_barrier pins the group order.
// hipcc-flags: -fno-slp-vectorize
// (the scale pass's f32 multiplies / FM sums beside the MFMAs: SLP packs them
// into v_pk_mul_f32 / v_pk_add_f32, which cost more MFMA-gap issue than pairs
// of scalar ops, MI355X_MICROARCH.md "price of one filler")
// MFMA: D = W_frag x X_frag^T: lane (r, h) = (l & 31, l >> 5) holds
// C[m = 32 im + r][n = 32 jn + (g & 3) + 8 (g >> 2) + 4 h] in register g.
#include <utility>

#include "asm_io.h"
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

// Diagnostic build only (tools/native/gg1w_stamps.hip defines it): s_memtime
// stamps of one K tile in the middle of the loop (after the barrier, after
// steps 0, 3, 4, 5, 6, 7) plus entry / prologue / loop / epilogue, kept in
// registers and written by lane 0 of each wave at the end.
#ifdef DTFS_GG1W_STAMPS
__device__ unsigned long long g_gg1w_stamps[4096][4][12];
#define G1_T(k)                                             \
  do {                                                      \
    if (t == g1_t) g1_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define G1_AT(k)                              \
  do {                                        \
    g1_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define G1_T(k) \
  do {          \
  } while (0)
#define G1_AT(k) \
  do {           \
  } while (0)
#endif

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {
template <int N>
__device__ __forceinline__ void wait_lgkm4(bf16x8 (&x)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_lgkm_q(bf16x8& a, bf16x8& b, bf16x8& c, bf16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_vm4(bf16x8 (&x)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N));
}
template <int OFF>
__device__ __forceinline__ bf16x8 lds_read16_at(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ i32x4 lds_read16i_at(uint32_t addr) {
  i32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ int lds_read4_at(uint32_t addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ void lds_write16_at(uint32_t addr, const i32x4& v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(addr), "v"(v), "n"(OFF) : "memory");
}
template <class Fn, int... I>
__device__ __forceinline__ void sfor_(Fn&& fn, std::integer_sequence<int, I...>) {
  (fn(std::integral_constant<int, I>{}), ...);
}
// fn(integral_constant<int, 0>) .. fn(integral_constant<int, N-1>): compile-time
// indices (LDS immediate offsets) in unrolled code
template <int N, class Fn>
__device__ __forceinline__ void sfor(Fn&& fn) {
  sfor_(fn, std::make_integer_sequence<int, N>{});
}
}  // namespace

template <bool FM>
__global__ void __launch_bounds__(256, 1) gemm_gather1w_kernel(const uint8_t* __restrict__ table, int Vm1,
                                                               const int32_t* __restrict__ rows_t,
                                                               const float* __restrict__ wts_t, int64_t Mp,
                                                               const bf16x8* __restrict__ Wp,
                                                               const float* __restrict__ bias, bf16* __restrict__ C,
                                                               int64_t ldc, float* __restrict__ fm_part, int M, int N,
                                                               int F, int relu) {
  constexpr int BM = 128, BN = 512;
  constexpr int NS = 4;   // A ring slots: tile t+1 (scale pass, then fragments), t+2 / t+3 (DMA), t (free)
  constexpr int RI = 8;   // rows / weights ring slots
  constexpr int LR = 6;   // ring lead (tiles)
  constexpr int SLOT = BM * 128;
  constexpr int RING = 1024;       // per tile: 128 int32 table rows | 128 fp32 weights
  constexpr int SP = BN * 2 + 16;  // epilogue staging pitch (bytes)
  constexpr int KLOOP = NS * SLOT + RI * RING;
  constexpr int SMEM = BM * SP > KLOOP ? BM * SP : KLOOP;
#ifdef DTFS_GG1W_STAMPS
  unsigned long long g1_s[12] = {};
  const int g1_t = F / 2;
#endif
  G1_AT(0);
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  uint8_t* const rring = smem + NS * SLOT;
  const uint32_t aring_lds = lds_addr(smem);
  const uint32_t rring_lds = lds_addr(rring);

  const int tiles_n = N / BN, tiles_m = int(Mp / BM);
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile % tiles_n;  // N-fastest: a row tile's column tiles share an XCD
  const int m0 = tm * BM, n0 = tn * BN;
  const int T = threadIdx.x;
  const int lane = T & 63;
  const int w = __builtin_amdgcn_readfirstlane(T >> 6);
  const int r32 = lane & 31, h = lane >> 5;

  // ---- staging (VMEM: every wave issues the same number per tile)
  auto stage_ring = [&](int u) {  // 1 op: lanes 0-31 the rows, 32-63 the weights of tile u
    const int uc = min(u, F - 1);
    const void* g = lane < 32 ? static_cast<const void*>(rows_t + int64_t(uc) * Mp + m0 + 4 * lane)
                              : static_cast<const void*>(wts_t + int64_t(uc) * Mp + m0 + 4 * (lane - 32));
    lds_dma16(g, rring_lds + (u & (RI - 1)) * RING);
  };
  // A tile u: wave w DMAs rows R = 32 w + 8 k + (lane >> 3), k = 0..3 (1 KiB
  // each); lane i lands at +16 i = physical chunk lane & 7 of row R, which
  // holds logical chunk (lane & 7) ^ (R & 7)  (swizzle: chunk ^ (row & 7))
  const int arow0 = 32 * w + (lane >> 3);
  const int a_src = ((lane & 7) ^ ((lane >> 3) & 7)) << 4;
  const uint32_t aring_w = aring_lds + 32 * w * 128;
  const uint32_t idx_off = 4 * arow0;
  int aidx[4];
  auto read_idx = [&](int u) {  // 4 LDS ops
    const uint32_t base = rring_lds + (u & (RI - 1)) * RING + idx_off;
    sfor<4>([&](auto k) { aidx[k] = lds_read4_at<32 * k>(base); });
  };
  auto stage_a = [&](int u, int k) {  // 1 op; aidx of tile u landed (table < 4 GiB: a 32-bit offset)
    const int rr = min(max(aidx[k], 0), Vm1);
    lds_dma16_s(table, uint32_t(rr) * 128u + a_src, aring_w + (u & (NS - 1)) * SLOT + k * 1024);
  };
  // W fragments of wave w (the MFMA's A operand, 32 columns x 16 K each):
  // packed blocks n0 / 32 + 4 w + jn, layout [N/32][F][4][64][8] (ops.pack_frag32)
  // (the fragment's address is uniform but for the lane's 16 bytes: SGPR base)
  const bf16x8* wpw = Wp + int64_t(n0 / 32 + 4 * w) * F * 4 * 64;
  const uint32_t w_lane = 16 * lane;
  bf16x8 wf[4][4];
  auto load_w1 = [&](int u, int jn, int s) {  // 1 op
    wf[jn][s] = gload16_s(wpw + ((int64_t(jn) * F + min(u, F - 1)) * 4 + s) * 64, w_lane);
  };

  // ---- x fragments (the MFMA's B operand): row 32 im + r32, K 16 s + 8 h ..
  // +7 = logical chunk 2 s + h, physical (2 s + h) ^ (r32 & 7)
  bf16x8 xf[4][4];
  // chunk (2 s + h) ^ (r32 & 7) = ((h ^ (r32 & 1)) | 2 (s ^ ((r32 >> 1) & 3))):
  // bits 5-6 of the byte offset are s ^ ((r32 >> 1) & 3), so one register
  // holds the s = 0 offset and K step s XORs (s << 5) into it
  const uint32_t xo0 = r32 * 128 + ((h ^ (r32 & 1)) << 4) + (((r32 >> 1) & 3) << 5);
  auto read_xs = [&](int u, int s) {  // 4 ops: K step s of all 4 row blocks
    const uint32_t a = aring_lds + (u & (NS - 1)) * SLOT + (xo0 ^ uint32_t(s << 5));
    sfor<4>([&](auto im) { xf[im][s] = lds_read16_at<4096 * im>(a); });
  };
  // ---- scale pass: thread T rescales logical chunk T & 7 of rows (T >> 3) +
  // 32 ((q + qrot) & 3), q = 0..3. DeepFM: column tile tn owns the FM term of
  // rows 64 tn .. 64 tn + 63 (tn < 2), rotated to q = 0, 1 so that the FM sums
  // are straight-line code (a branch would split the scheduling region and keep
  // the scale pass's VALU from interleaving with the MFMAs).
  const int sc_c = T & 7, sc_r0 = T >> 3;
  const uint32_t sc_off = sc_r0 * 128 + ((sc_c ^ (sc_r0 & 7)) << 4);
  const int qrot = FM ? 2 * tn : 0;
  auto qq = [&](int q) { return (q + qrot) & 3; };
  i32x4 sv[4];
  int swt[4];
  float fs[2][8], fsq[2] = {0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int d = 0; d < 8; ++d) fs[a][d] = 0.f;
  auto scale_read = [&](int u) {  // 8 ops
    const uint32_t base = aring_lds + (u & (NS - 1)) * SLOT + sc_off;
    const uint32_t wb = rring_lds + (u & (RI - 1)) * RING + 512 + 4 * sc_r0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sv[q] = lds_read16i_at<0>(base + 4096 * qq(q));
      swt[q] = lds_read4_at<0>(wb + 128 * qq(q));
    }
  };
  auto scale_wait = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(sv[0]), "+v"(sv[1]), "+v"(sv[2]), "+v"(sv[3]), "+v"(swt[0]), "+v"(swt[1]), "+v"(swt[2]),
                   "+v"(swt[3]));
  };
  // one bf16 pair of chunk q (5 VALU, + 4 for the FM sums): the unit the
  // steps interleave with their MFMAs; pair 3 writes the chunk back (1 op)
  i32x4 so[4];
  auto scale_pair = [&](int u, int q, int p) {
    // u == F: the trailing re-staged tile (never multiplied): zero weight, so
    // the FM sums stay exact without a branch
    const float wt = u < F ? __int_as_float(swt[q]) : 0.f;
    const float a = __uint_as_float(uint32_t(sv[q][p]) << 16) * wt;
    const float b = __uint_as_float(uint32_t(sv[q][p]) & 0xffff0000u) * wt;
    so[q][p] = __builtin_bit_cast(int, __builtin_convertvector((f32x2){a, b}, bf16x2));
    if constexpr (FM) {
      if (q < 2) {  // compile-time after unrolling
        fs[q][2 * p] += a;
        fs[q][2 * p + 1] += b;
        fsq[q] += a * a;
        fsq[q] += b * b;
      }
    }
    if (p == 3) lds_write16_at<0>(aring_lds + (u & (NS - 1)) * SLOT + sc_off + 4096 * qq(q), so[q]);
  };
  auto scale_write = [&](int u, int q) {
#pragma unroll
    for (int p = 0; p < 4; ++p) scale_pair(u, q, p);
  };

  f32x16 acc[4][4];  // [jn][im]: D[n = 32 jn + (g & 3) + 8 (g >> 2) + 4 h][m = 32 im + r32]
#pragma unroll
  for (int jn = 0; jn < 4; ++jn)
#pragma unroll
    for (int im = 0; im < 4; ++im)
#pragma unroll
      for (int g = 0; g < 16; ++g) acc[jn][im][g] = 0.f;
  // MFMA groups run K step s over the 4 row blocks; a group's operands are
  // only overwritten (next tile's loads) a whole group later: an in-flight
  // MFMA can still be reading its source registers, and the loads are inline
  // asm the hazard recognizer does not pad
  auto group = [&](int jn, int s) {
#pragma unroll
    for (int im = 0; im < 4; ++im)
      acc[jn][im] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[jn][s], xf[im][s], acc[jn][im], 0, 0, 0);
  };
  auto mfma1 = [&](int jn, int im, int s) {
    acc[jn][im] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[jn][s], xf[im][s], acc[jn][im], 0, 0, 0);
  };
  auto fence = [] { __builtin_amdgcn_sched_barrier(0); };
#define WAIT_XS(N, s) wait_lgkm_q<N>(xf[0][s], xf[1][s], xf[2][s], xf[3][s])
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto wait_idx = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aidx[0]), "+v"(aidx[1]), "+v"(aidx[2]), "+v"(aidx[3])::"memory");
  };

  // ---- VMEM: per tile t, four load groups, each issued one op per MFMA pair
  // inside the step after the one that last read its registers:
  //   G3(t-1) in step 0: W(t, 3) x 4, ring(t + 5)
  //   G0(t)   in step 1: W(t+1, 0) x 4, A(t+3, 0..1)
  //   G1(t)   in step 2: W(t+1, 1) x 4, A(t+3, 2..3)
  //   G2(t)   in step 3: W(t+1, 2) x 4
  // so the counted wait for W(t, jn) at the top of step jn is vmcnt 12, 11, 11,
  // 13 (the ops issued after it, in order). vmcnt retires in issue order:
  // step 2's wait retires G1(t-1) (A(t+2)) before the tile's barrier, step 1's
  // retires G3(t-1) (ring(t+5)) long before read_idx(t+5) at tile t+1.
  auto vm_op = [&](int t, int g, int i) {
    if (g == 3) {
      if (i < 4) load_w1(t, 3, i);
      else stage_ring(t + 5);
    } else if (i < 4) {
      load_w1(t + 1, g, i);
    } else {
      stage_a(t + 3, 2 * g + (i - 4));
    }
  };

  // ---- prologue: rings 0..4; A(0), A(1); then G0(-1), G1(-1), G2(-1) in the
  // loop's order, so the loop's counted waits hold from the first tile on;
  // A(0) scaled; idx(3) read; K steps 0-2 of A(0)'s fragments in flight as
  // step 3 of a tile leaves them
  for (int u = 0; u < LR - 1; ++u) stage_ring(u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  read_idx(0);
  wait_idx();
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(0, k);
  read_idx(1);
  wait_idx();
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(1, k);
  read_idx(2);
  wait_idx();
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int i = 0; i < (g == 2 ? 4 : 6); ++i) vm_op(-1, g, i);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // A(0), A(1) landed (this wave's share)
  barrier();
  scale_read(0);
  scale_wait();
#pragma unroll
  for (int q = 0; q < 4; ++q) scale_write(0, q);
  read_idx(3);
  wait_idx();
  barrier();
  read_xs(0, 0);
  read_xs(0, 1);
  read_xs(0, 2);

  G1_AT(1);
  // ---- main loop: K tile t = field t, 4 steps (column blocks jn of 32), 16
  // MFMAs (K steps s-major over the 4 row blocks) each, issued in pairs; a
  // pair carries one VMEM op and / or one bf16 pair of the scale pass.
  // LDS per tile: step 0 waits for A(t)'s fragments (K steps 0-2 read during
  // step 3 of tile t-1, K step 3 after step 0's first group: lgkmcnt 8, 8, 4,
  // 0 per K step), and reads A(t+1) for the scale pass, whose 4 writes go out
  // during steps 1-2; step 2 reads idx(t+4) after its last A DMA, then
  // lgkmcnt(0) + the tile's one barrier; step 3 reads K steps 0-2 of A(t+1)'s
  // fragments (at most 12 LDS ops outstanding: lgkmcnt is a 4-bit counter).
  // Hazards (slots mod 4): the barrier of tile t-1 follows that tile's step-2
  // wait, which retired A(t+1)'s DMAs (G0 / G1 of tile t-2): the scale pass
  // reads them after it. The scale writes of tile t+1 precede tile t's
  // barrier; its fragments are read after it. A(t+3) (steps 1-2) overwrites
  // slot t-1, whose last fragments were read at step 0 of tile t-1.
  // Every wave DMAs the same ring bytes: its own DMA having landed is enough
  // to read them.
#pragma unroll 1
  for (int t = 0; t < F; ++t) {
    auto pair = [&](int jn, int k) {
      mfma1(jn, (2 * k) & 3, k >> 1);
      mfma1(jn, (2 * k + 1) & 3, k >> 1);
    };
    if constexpr (FM) {
      // the FM sums are complete once tile F-1 is scaled (during tile F-2):
      // the last tile stores the partials, so none of their registers live
      // past the loop (there the allocator spilled accumulators to scratch)
      if (t == F - 1) {
        const int sc_ce = T & 7, sc_r0e = T >> 3;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          float part = -fsq[a];
#pragma unroll
          for (int d = 0; d < 8; ++d) part += fs[a][d] * fs[a][d];
          part += __shfl_xor(part, 1, 64);
          part += __shfl_xor(part, 2, 64);
          part += __shfl_xor(part, 4, 64);
          if (tn < 2 && sc_ce == 0) fm_part[Mp + m0 + sc_r0e + 32 * (2 * tn + a)] = 0.5f * part;
        }
        // the shuffles are LDS ops the compiler tracks: retire them here, or
        // it drains lgkmcnt in the middle of step 0 on every tile
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      }
    }
    // step 0: A(t)'s fragments land K step by K step; G3(t-1)
    wait_vm4<12>(wf[0]);
    G1_T(2);
    WAIT_XS(8, 0);
    pair(0, 0);
    fence();
    pair(0, 1);
    vm_op(t, 3, 0);
    fence();
    read_xs(t, 3);  // registers last read by step 3 of tile t-1
    WAIT_XS(8, 1);
    pair(0, 2);
    vm_op(t, 3, 1);
    fence();
    pair(0, 3);
    vm_op(t, 3, 2);
    fence();
    WAIT_XS(4, 2);
    pair(0, 4);
    vm_op(t, 3, 3);
    fence();
    pair(0, 5);
    vm_op(t, 3, 4);
    fence();
    WAIT_XS(0, 3);
    scale_read(t + 1);
    pair(0, 6);
    fence();
    pair(0, 7);
    fence();
    G1_T(3);
    // step 1: the scale pass's chunks 0-1, one bf16 pair per MFMA pair; G0(t)
    wait_vm4<11>(wf[1]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(1, k);
      if (k == 0) scale_wait();  // the scale reads had step 0's last two pairs + this one
      scale_pair(t + 1, k >> 2, k & 3);
      if (k >= 1 && k <= 6) vm_op(t, 0, k - 1);
      fence();
    }
    G1_T(4);
    // step 2: chunks 2-3; G1(t); then the rows of A(t+4)
    wait_vm4<11>(wf[2]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pair(2, k);
      scale_pair(t + 1, 2 + (k >> 2), k & 3);
      if (k >= 1 && k <= 6) vm_op(t, 1, k - 1);
      if (k == 7) read_idx(t + 4);
      fence();
    }
    G1_T(5);
    wait_idx();  // + this wave's scale writes
    barrier();
    G1_T(6);
    // step 3: K steps 0-2 of A(t+1) stream in, each a group after its
    // registers' last use; G2(t)
    wait_vm4<13>(wf[3]);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k == 4) read_xs(t + 1, 0);
      if (k == 6) read_xs(t + 1, 1);
      pair(3, k);
      if (k >= 1 && k <= 4) vm_op(t, 2, k - 1);
      fence();
    }
    read_xs(t + 1, 2);
    G1_T(7);
    G1_T(8);
  }
  G1_AT(9);
#undef WAIT_XS
  // the trailing (re-staged, unread) loads land before the LDS is reused / the waves exit
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // nothing of the tail above the wait: the registers of the dead trailing
  // prefetches are free to the compiler after the loop (see cross_gemm.hip)
  __builtin_amdgcn_sched_barrier(0);
  // Lane-derived indices of the tail are recomputed here from a volatile read
  // of the lane id (not CSE'd with the prologue's): kept live across the loop,
  // the register allocator spilled them to scratch - and a scratch-using
  // kernel faulted (memory aperture violation) once captured into the served
  // step's HIP graph. Scratch-free is checked by test_kernels_gpu.
  int lane_e;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
  int tid_e;
  asm volatile("v_mov_b32 %0, %1" : "=v"(tid_e) : "v"(lane_e));
  tid_e += 64 * w;
  const int r32e = lane_e & 31, he = lane_e >> 5, sc_ce = tid_e & 7, sc_r0e = tid_e >> 3;
  __syncthreads();

  // ---- epilogue: bias + act -> bf16, staged through LDS, written as whole 1 KiB rows
  {
    const float lo = relu ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int jn = 0; jn < 4; ++jn) {
      f32x4 b4[4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
        b4[g4] = *reinterpret_cast<const f32x4*>(bias + n0 + 128 * w + 32 * jn + 8 * g4 + 4 * he);
#pragma unroll
      for (int im = 0; im < 4; ++im) {
        // a whole 16-register accumulator at a time (sub-register pieces made
        // the allocator shuffle AGPRs at the loop exit, through scratch)
        const f32x16 av = acc[jn][im];
        const int m = 32 * im + r32e;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int n = 128 * w + 32 * jn + 8 * g4 + 4 * he;
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = f2bf(fmaxf(av[4 * g4 + e] + b4[g4][e], lo));
          *reinterpret_cast<bf16x4*>(smem + m * SP + n * 2) = o;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int r = w; r < BM; r += 4) {
    const int m = m0 + r;
    if (m < M)
      *reinterpret_cast<bf16x8*>(C + int64_t(m) * ldc + n0 + 8 * lane_e) =
          *reinterpret_cast<const bf16x8*>(smem + r * SP + 16 * lane_e);
  }
#ifdef DTFS_GG1W_STAMPS
  G1_AT(10);
  if (lane_e == 0 && blockIdx.x < 4096)
    for (int k = 0; k < 12; ++k) g_gg1w_stamps[blockIdx.x][w][k] = g1_s[k];
#endif
}

}  // namespace kern

bool gemm_gather1w_ok(int64_t Mp, int N, int F, bool cross, int64_t V) {
  // V <= 2^25: table row offsets (128 B rows) fit the 32-bit DMA offset
  return !cross && N % 512 == 0 && Mp % 128 == 0 && F >= 1 && F <= 4096 && V >= 1 && V <= (int64_t(1) << 25);
}

hipError_t launch_gemm_gather1w(const void* table, int64_t V, const int32_t* rows_t, const float* wts_t, int64_t Mp,
                                int F, const void* Wp, const float* bias, void* C, int64_t ldc, float* fm_part, int M,
                                int N, int epi, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (!gemm_gather1w_ok(Mp, N, F, false, V) || Mp < M || ldc < N || ldc % 8 != 0 ||
      (fm_part && N < 1024) || !table || !rows_t || !wts_t || !Wp || !C || !bias)
    return hipErrorInvalidValue;
  const int grid = int(Mp / 128) * (N / 512);
  const int relu = (epi & 15) == 1;
  if (fm_part)
    hipLaunchKernelGGL((kern::gemm_gather1w_kernel<true>), dim3(grid), dim3(256), 0, st,
                       static_cast<const uint8_t*>(table), int(V - 1), rows_t, wts_t, Mp,
                       static_cast<const kern::bf16x8*>(Wp), bias, static_cast<kern::bf16*>(C), ldc, fm_part, M, N,
                       F, relu);
  else
    hipLaunchKernelGGL((kern::gemm_gather1w_kernel<false>), dim3(grid), dim3(256), 0, st,
                       static_cast<const uint8_t*>(table), int(V - 1), rows_t, wts_t, Mp,
                       static_cast<const kern::bf16x8*>(Wp), bias, static_cast<kern::bf16*>(C), ldc, nullptr, M, N,
                       F, relu);
  return hipGetLastError();
}

}  // namespace dtfs

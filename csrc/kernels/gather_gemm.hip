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
//     all 128 rows (acc 8 x 8 16x16 blocks = 256 registers);
//   * B (W1) never touches LDS: it is kept in MFMA fragment order
//     (ops.pack_bfrag) and each wave loads its own fragments straight into
//     registers, one K tile ahead, rolling: B(t+1, j) refills the registers of
//     B(t, j) right after column block j's MFMAs (MFMA order: column block j
//     outer, row block i inner);
//   * A (the gathered table rows, 128 x 128 B per field) goes through a 6-slot
//     LDS ring by LDS-DMA, three K tiles ahead of its MFMAs; the weights are
//     applied ONCE per element in LDS by a scale pass over tile t+1 while tile
//     t's MFMAs run (the unfused gather's bf16(w * e) rounding, bit for bit),
//     which also accumulates the FM sums;
//   * one barrier per K tile; every vmcnt / lgkmcnt is counted (all hot-loop
//     memory operations are inline asm, csrc/kernels/asm_io.h).
// MFMA: v_mfma_f32_16x16x32_bf16 in the transposed form (D = W_frag x A_frag^T:
// lane (fr, fq) holds C[m = fr][n = 4 fq .. +3]).
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

namespace {
template <int N>
__device__ __forceinline__ void wait_lgkm(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_lgkm_idx(bf16x8& a, bf16x8& b, int (&x)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(a), "+v"(b), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(N));
}
template <int N>
__device__ __forceinline__ void wait_vm(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N));
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
  constexpr int NS = 6;   // A ring slots: tile t (MFMA), t+1 (scale), t+2 / t+3 (DMA in flight), 2 spare
  constexpr int RI = 8;   // rows / weights ring slots
  constexpr int LR = 6;   // ring lead (tiles)
  constexpr int SLOT = BM * 128;
  constexpr int RING = 1024;      // per tile: 128 int32 table rows | 128 fp32 weights
  constexpr int SP = BN * 2 + 16; // epilogue staging pitch (bytes)
  constexpr int KLOOP = NS * SLOT + RI * RING;
  constexpr int SMEM = BM * SP > KLOOP ? BM * SP : KLOOP;
#ifdef DTFS_GG1W_STAMPS
  unsigned long long g1_s[12] = {};
  const int g1_t = F / 2;
#endif
  G1_AT(0);
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  uint8_t* const aring = smem;
  uint8_t* const rring = smem + NS * SLOT;

  const int tiles_n = N / BN, tiles_m = int(Mp / BM);
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile % tiles_n;  // N-fastest: a row tile's column tiles share an XCD
  const int m0 = tm * BM, n0 = tn * BN;
  const int T = threadIdx.x;
  const int lane = T & 63;
  const int w = __builtin_amdgcn_readfirstlane(T >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // ---- staging helpers (VMEM: every wave issues the same number per tile)
  const uint32_t rring_lds = lds_addr(rring);
  auto stage_ring = [&](int u) {  // 1 op: lanes 0-31 the rows, 32-63 the weights of tile u
    const int uc = min(u, F - 1);
    const void* g = lane < 32 ? static_cast<const void*>(rows_t + int64_t(uc) * Mp + m0 + 4 * lane)
                              : static_cast<const void*>(wts_t + int64_t(uc) * Mp + m0 + 4 * (lane - 32));
    lds_dma16(g, rring_lds + (u & (RI - 1)) * RING);
  };
  // A tile u: wave w DMAs rows 32 w + 8 k + (lane >> 3), k = 0..3 (1 KiB each;
  // lane i lands at +16 i, so its source is the logical chunk that swizzles there)
  const int arow0 = 32 * w + (lane >> 3);
  const uint32_t aring_w = lds_addr(aring) + 32 * w * 128;
  int aidx[4];
  auto read_idx = [&](int u) {  // 4 LDS ops
    const int32_t* ri = reinterpret_cast<const int32_t*>(rring + (u & (RI - 1)) * RING);
#pragma unroll
    for (int k = 0; k < 4; ++k) aidx[k] = lds_read4(ri + arow0 + 8 * k);
  };
  auto stage_a = [&](int u, int k) {  // 1 op; aidx of tile u landed
    const int R = arow0 + 8 * k;
    const int r = min(max(aidx[k], 0), Vm1);
    const uint8_t* g = table + int64_t(r) * 128 + (((lane & 7) ^ ((R >> 1) & 7)) << 4);
    lds_dma16(g, aring_w + (u % NS) * SLOT + k * 1024);
  };
  // B fragments of wave w: packed blocks n0 / 16 + 8 w + j, layout [N/16][F][2][64][8]
  const bf16x8* wpw = Wp + int64_t(n0 / 16 + 8 * w) * F * 2 * 64 + lane;
  bf16x8 b[8][2];
  auto load_b = [&](int u, int j) {  // 2 ops
    const int uc = min(u, F - 1);
    b[j][0] = gload16(wpw + ((int64_t(j) * F + uc) * 2 + 0) * 64);
    b[j][1] = gload16(wpw + ((int64_t(j) * F + uc) * 2 + 1) * 64);
  };

  // ---- LDS readers
  bf16x8 fa[8][2];
  auto read_a = [&](int u, int i) {  // 2 ops: rows 16 i + fr, logical chunks fq / 4 + fq
    const uint8_t* s = aring + (u % NS) * SLOT;
    const int row = 16 * i + fr;
    const int sw = (row >> 1) & 7;
    fa[i][0] = lds_read16(s + row * 128 + ((fq ^ sw) << 4));
    fa[i][1] = lds_read16(s + row * 128 + (((4 + fq) ^ sw) << 4));
  };
  // scale pass: thread T rescales logical chunk T & 7 of rows (T >> 3) + 32 q
  const int sc_c = T & 7;
  i32x4 sv[4];
  int swt[4];
  const bool fm_on = FM && fm_part != nullptr && tn < 2;  // column tile tn owns FM rows 64 tn .. 64 tn + 63
  float fs[2][8], fsq[2] = {0.f, 0.f};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int d = 0; d < 8; ++d) fs[a][d] = 0.f;
  auto scale_row = [&](int q) { return (T >> 3) + 32 * q; };
  auto scale_addr = [&](int u, int q) {
    const int row = scale_row(q);
    return aring + (u % NS) * SLOT + row * 128 + ((sc_c ^ ((row >> 1) & 7)) << 4);
  };
  auto scale_read = [&](int u) {  // 8 ops
    const float* wr = reinterpret_cast<const float*>(rring + (u & (RI - 1)) * RING + 512);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      sv[q] = lds_read16i(scale_addr(u, q));
      swt[q] = lds_read4(wr + scale_row(q));
    }
  };
  auto scale_wait = [&] {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(sv[0]), "+v"(sv[1]), "+v"(sv[2]), "+v"(sv[3]), "+v"(swt[0]), "+v"(swt[1]), "+v"(swt[2]),
                   "+v"(swt[3]));
  };
  auto scale_write = [&](int u, int q) {  // 1 op
    const float wt = __int_as_float(swt[q]);
    i32x4 o;
    float v[8];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      v[2 * p] = __uint_as_float(uint32_t(sv[q][p]) << 16) * wt;
      v[2 * p + 1] = __uint_as_float(uint32_t(sv[q][p]) & 0xffff0000u) * wt;
      int r;
      asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(v[2 * p]), "v"(v[2 * p + 1]));
      o[p] = r;
    }
    lds_write16(scale_addr(u, q), o);
    if constexpr (FM) {
      if (fm_on && (q >> 1) == tn && u < F) {  // u == F: the trailing re-staged tile
#pragma unroll
        for (int d = 0; d < 8; ++d) {
          fs[q & 1][d] += v[d];
          fsq[q & 1] += v[d] * v[d];
        }
      }
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfma_col = [&](int j) {  // column block j x all 8 row blocks
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][kk], fa[i][kk], acc[i][j], 0, 0, 0);
  };
  auto mfma_blk = [&](int i) {  // column block 0 x row block i (step 0, while A streams in)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[0][kk], fa[i][kk], acc[i][0], 0, 0, 0);
  };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- prologue: rings 0..LR-1; A(0), A(1); then "tile -1" in the loop's VMEM order
  // (B(0, j) x 2, A(2, j) for j < 4, a ring op at j = 4: 21 ops), so the loop's
  // counted waits hold from the first tile on
  for (int u = 0; u < LR; ++u) stage_ring(u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  read_idx(0);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aidx[0]), "+v"(aidx[1]), "+v"(aidx[2]), "+v"(aidx[3]));
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(0, k);
  read_idx(1);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aidx[0]), "+v"(aidx[1]), "+v"(aidx[2]), "+v"(aidx[3]));
#pragma unroll
  for (int k = 0; k < 4; ++k) stage_a(1, k);
  read_idx(2);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(aidx[0]), "+v"(aidx[1]), "+v"(aidx[2]), "+v"(aidx[3]));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    load_b(0, j);
    if (j < 4) stage_a(2, j);
    if (j == 4) stage_ring(LR - 1);  // the ring op of "tile -1" (same bytes again)
  }
  asm volatile("s_waitcnt vmcnt(21)" ::: "memory");  // A(0) landed (this wave's share)
  barrier();
  scale_read(0);
  scale_wait();
#pragma unroll
  for (int q = 0; q < 4; ++q) scale_write(0, q);

  G1_AT(1);
  // ---- main loop: K tile t = field t
  // VMEM per tile (per wave, in order): step j: B(t+1, j) x 2, then A(t+3, j)
  // (j < 4) or ring(t + LR) (j == 4): 21 ops. Before step j's MFMAs, B(t, j)
  // (issued at step j of tile t-1) has exactly 19 newer ops: vmcnt(19). That
  // wait at step 0 also retires every op of tile t-2: A(t+1) (scale pass of
  // this tile) and ring(t+3) (read_idx below, after the barrier).
  // LDS per tile: A(t) blocks 0-3, idx(t+3), blocks 4-7 during step 0, the
  // scale pass of tile t+1 (8 reads at step 4, 4 writes at steps 5-6).
  // Hazards (slots mod 6): A(t+3) is written after this tile's barrier, its
  // slot last read by tile t-3; the scale pass rewrites slot t+1 (landed for
  // every wave: vmcnt at step 0 + barrier) that nobody reads this tile; tile
  // t's fragments were scaled during tile t-1 (lgkmcnt(0) + barrier).
#pragma unroll 1
  for (int t = 0; t < F; ++t) {
    asm volatile("s_waitcnt vmcnt(19) lgkmcnt(0)" : "+v"(b[0][0]), "+v"(b[0][1])::"memory");
    barrier();
    G1_T(2);
#pragma unroll
    for (int i = 0; i < 4; ++i) read_a(t, i);
    read_idx(t + 3);
    // step 0: A fragments stream in (lgkmcnt per row block)
    wait_lgkm<10>(fa[0][0], fa[0][1]);
    mfma_blk(0);
    read_a(t, 4);
    wait_lgkm<10>(fa[1][0], fa[1][1]);
    mfma_blk(1);
    read_a(t, 5);
    wait_lgkm<10>(fa[2][0], fa[2][1]);
    mfma_blk(2);
    read_a(t, 6);
    wait_lgkm<10>(fa[3][0], fa[3][1]);
    mfma_blk(3);
    read_a(t, 7);
    wait_lgkm_idx<6>(fa[4][0], fa[4][1], aidx);
    mfma_blk(4);
    wait_lgkm<4>(fa[5][0], fa[5][1]);
    mfma_blk(5);
    wait_lgkm<2>(fa[6][0], fa[6][1]);
    mfma_blk(6);
    wait_lgkm<0>(fa[7][0], fa[7][1]);
    mfma_blk(7);
    load_b(t + 1, 0);
    stage_a(t + 3, 0);
    G1_T(3);
#pragma unroll
    for (int j = 1; j < 4; ++j) {
      wait_vm<19>(b[j][0], b[j][1]);
      mfma_col(j);
      load_b(t + 1, j);
      stage_a(t + 3, j);
    }
    G1_T(4);
    wait_vm<19>(b[4][0], b[4][1]);
    scale_read(t + 1);
    mfma_col(4);
    load_b(t + 1, 4);
    stage_ring(t + LR);
    G1_T(5);
    wait_vm<19>(b[5][0], b[5][1]);
    scale_wait();
    scale_write(t + 1, 0);
    scale_write(t + 1, 1);
    mfma_col(5);
    load_b(t + 1, 5);
    G1_T(6);
    wait_vm<19>(b[6][0], b[6][1]);
    scale_write(t + 1, 2);
    scale_write(t + 1, 3);
    mfma_col(6);
    load_b(t + 1, 6);
    G1_T(7);
    wait_vm<19>(b[7][0], b[7][1]);
    mfma_col(7);
    load_b(t + 1, 7);
    G1_T(8);
  }
  G1_AT(9);
  // the trailing (re-staged, unread) loads land before the LDS is reused / the waves exit
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: bias + act -> bf16, staged through LDS, written as whole 1 KiB rows
  {
    const float lo = relu ? 0.f : -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = 128 * w + 16 * j + 4 * fq;
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(bias + n0 + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = 16 * i + fr;
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc[i][j][r] + b4[r], lo));
        *reinterpret_cast<bf16x4*>(smem + m * SP + n * 2) = o;
      }
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int r = w; r < BM; r += 4) {
    const int m = m0 + r;
    if (m < M)
      *reinterpret_cast<bf16x8*>(C + int64_t(m) * ldc + n0 + 8 * lane) =
          *reinterpret_cast<const bf16x8*>(smem + r * SP + 16 * lane);
  }
#ifdef DTFS_GG1W_STAMPS
  G1_AT(10);
  if (lane == 0 && blockIdx.x < 4096)
    for (int k = 0; k < 12; ++k) g_gg1w_stamps[blockIdx.x][w][k] = g1_s[k];
#endif
  if constexpr (FM) {
    if (fm_on) {
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        float part = -fsq[a];
#pragma unroll
        for (int d = 0; d < 8; ++d) part += fs[a][d] * fs[a][d];
        part += __shfl_xor(part, 1, 64);
        part += __shfl_xor(part, 2, 64);
        part += __shfl_xor(part, 4, 64);
        if (sc_c == 0) fm_part[Mp + m0 + scale_row(2 * tn + a)] = 0.5f * part;
      }
    }
  }
}

}  // namespace kern

bool gemm_gather1w_ok(int64_t Mp, int N, int F, bool cross) {
  return !cross && N % 512 == 0 && Mp % 128 == 0 && F >= 1 && F <= 4096;
}

hipError_t launch_gemm_gather1w(const void* table, int64_t V, const int32_t* rows_t, const float* wts_t, int64_t Mp,
                                int F, const void* Wp, const float* bias, void* C, int64_t ldc, float* fm_part, int M,
                                int N, int epi, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (!gemm_gather1w_ok(Mp, N, F, false) || Mp < M || V < 1 || V > (int64_t(1) << 31) || ldc < N || ldc % 8 != 0 ||
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

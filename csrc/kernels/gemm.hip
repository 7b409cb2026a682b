// K3b/K4/K6: dense towers on CDNA4 matrix cores.
//
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] )       A: [M][K], W: [N][K]
//
// bf16 operands use v_mfma_f32_16x16x32_bf16; fp8 (OCP e4m3) operands use the
// block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales; 2x the
// plain fp8 MFMA rate) with a per-row activation scale and a per-output-channel
// weight scale folded into the epilogue.
//
// Structure (cdna_hip_programming.md §5 "standard MFMA GEMM main loop"):
//   * 256 threads = 4 waves in a 2x2 grid; wave tile (BM/2)x(BN/2) made of
//     16x16 MFMA tiles, accumulators in registers.
//   * K tile = 128 bytes per row (64 bf16 or 128 fp8): each row of an LDS tile is
//     8 x 16-byte chunks, stored XOR-swizzled (chunk ^ ((row>>1)&7)) so the
//     16 distinct rows a ds_read lane group touches land on 16 distinct 16-B
//     bank slots (two 128-B rows share a 256-B bank row).
//   * register-staged double buffer: the next K tile's global loads are issued
//     before the MFMAs of the current tile and written to the other LDS buffer
//     after them, one __syncthreads per K tile.
//   * XCD-aware tile order (common.h xcd_remap) so neighbouring tiles sharing a
//     W panel run on one L2.
// Epilogues: bias, ReLU, sigmoid, DCN-v2 cross (x0 * (acc + b) + xl), written
// as bf16 or fp32.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

typedef int i32x8 __attribute__((ext_vector_type(8)));  // 32 x e4m3, the block-scaled MFMA operand

enum Epi { EPI_NONE = 0, EPI_RELU = 1, EPI_SIGMOID = 2, EPI_CROSS = 3 };

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// fp8 K tile on the block-scaled MFMA: v_mfma_scale_f32_16x16x128_f8f6f4 with
// e4m3 operands and unit E8M0 block scales (127 = 2^0) runs at 2x the rate of
// the non-scaled v_mfma_f32_16x16x32_fp8_fp8 (which only matches bf16;
// cdna_hip_programming.md §3 "MFMA rate per dtype"), and one instruction
// covers the whole 128-byte K tile. The real scales (per activation row, per
// weight channel) stay in the fp32 epilogue. Lane l holds row l&15,
// k = 32*(l>>4) .. +31 = 16-B chunks 2*(l>>4) and 2*(l>>4)+1 of the row.
// Operand layout of the 16x16x128 f8f6f4 MFMA (measured, bench_native/mx_probe.hip):
// lane (r = l & 15, q = l >> 4) holds row r, K [16q, 16q + 16) in its first 4
// VGPRs and K [64 + 16q, 64 + 16q + 16) in the last 4; the scale operand of
// lane (r, q) scales row r's K block [32q, 32q + 32). Loading 16-byte chunks q
// and q + 4 of the 128-byte K row keeps logical K = hardware K, so the MX
// block scales line up (any common permutation would do for unscaled use).
__device__ __forceinline__ i32x8 mx_frag(const uint8_t* tile, int row, int fq) {
  const i32x4 lo = *reinterpret_cast<const i32x4*>(tile + swz(row, fq));
  const i32x4 hi = *reinterpret_cast<const i32x4*>(tile + swz(row, fq + 4));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ f32x4 mx_mfma(const i32x8& a, const i32x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// Same with a real E8M0 block scale for the b operand (the activation
// fragment: lane l holds row l&15, K block l>>4, and supplies that block's
// scale byte; OCP MX: value = e4m3 x 2^(scale - 127)).
__device__ __forceinline__ f32x4 mx_mfma_sb(const i32x8& a, const i32x8& b, const f32x4& c, int scale_b) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, scale_b);
}

// Every kernel below issues its MFMAs as D = W_frag x A_frag^T, i.e. it
// computes the TRANSPOSED 16x16 output tile: with the C/D layout (col =
// lane & 15, row = 4 * (lane >> 4) + r) a lane then holds C[m = fr][n = 4 fq
// .. 4 fq + 3] - four consecutive output columns of one row. The epilogue
// reads bias / scales / x0 / xl and writes C as 8- or 16-byte vectors per lane
// instead of 2- or 4-byte scalars (the DCN-v2 cross epilogue touches three
// [M, N] bf16 tensors).
// GEMM epilogue: scales, bias, activation / DCN-v2 cross, bf16 or fp32 store.
// Written so that the 32-tile unrolled 8-phase epilogue stays small and the
// accumulators stay in registers:
//  * one code path for every activation, selected by wave-uniform values
//    (relu = max with 0 vs -inf; sigmoid / cross = uniform branches). A
//    runtime switch INSIDE the unrolled tile loops made the 8-phase kernel's
//    epilogue ~15k straight-line instructions (instruction-cache bound, 14-19
//    us per block, bench_native/g8ph_stamps.hip); a switch around per-activation
//    copies spilled the accumulators to scratch (528 B/lane).
//  * every operand load (bias, scales, x0, xl) is issued ahead of its use
//    (clamped in-bounds addresses; only the stores are predicated), not one
//    load -> use -> store latency per tile.
template <bool FP8, bool RAGGED = true, int TM, int TN, typename OutT>
__device__ __forceinline__ void store_acc_t(const f32x4 (&acc)[TM][TN], int mb, int nb, int fr, int fq, int M, int N,
                                            const float* __restrict__ bias, const float* __restrict__ sa,
                                            const float* __restrict__ sw, OutT* __restrict__ C, int64_t ldc,
                                            const bf16* __restrict__ X0, const bf16* __restrict__ XL, int64_t ldx,
                                            int epi) {
  const int e = epi & 15;
  const bool cross = e == EPI_CROSS, sig = e == EPI_SIGMOID;
  const float lo = e == EPI_RELU ? 0.f : -__builtin_huge_valf();
  if (!RAGGED || ((N | int(ldc) | int(ldx)) & 3) == 0) {  // N % 4 == 0: a lane's 4 columns exist together
    // column-tile outer: per j one bias / scale vector, then every row tile's
    // operand loads are issued before the first use (few live registers)
    // every bias / scale vector of the tile is loaded before the first use:
    // one memory round trip for the epilogue instead of one per column tile
    // (tools/native/g8ph_stamps: the 8-phase epilogue took 6.3-8.8 us per
    // 256x256 tile with the loads inside the column loop)
    float sam[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) sam[i] = (FP8 && sa) ? sa[min(mb + i * 16 + fr, M - 1)] : 1.f;
    f32x4 b4v[TN], s4v[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nc = min(nb + j * 16 + fq * 4, N - 4);
      b4v[j] = bias ? *reinterpret_cast<const f32x4*>(bias + nc) : f32x4{0.f, 0.f, 0.f, 0.f};
      s4v[j] = f32x4{1.f, 1.f, 1.f, 1.f};
      if constexpr (FP8) {
        if (sw) s4v[j] = *reinterpret_cast<const f32x4*>(sw + nc);
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = nb + j * 16 + fq * 4;
      const int nc = min(n, N - 4);
      const f32x4 b4 = b4v[j];
      const f32x4 s4 = s4v[j];
      bf16x4 x0[TM], xl[TM];
      if (cross) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int64_t mc = min(mb + i * 16 + fr, M - 1);
          x0[i] = *reinterpret_cast<const bf16x4*>(X0 + mc * ldx + nc);
          xl[i] = *reinterpret_cast<const bf16x4*>(XL + mc * ldx + nc);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + fr;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = acc[i][j][r];
          if constexpr (FP8) x *= s4[r] * sam[i];
          v[r] = fmaxf(x + b4[r], lo);
        }
        if (sig) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = sigmoidf(v[r]);
        }
        if (cross) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = bf2f(x0[i][r]) * v[r] + bf2f(xl[i][r]);
        }
        if (m >= M || n >= N) continue;
        if constexpr (sizeof(OutT) == 2) {
          bf16x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
          *reinterpret_cast<bf16x4*>(C + int64_t(m) * ldc + n) = o;
        } else {
          *reinterpret_cast<f32x4*>(C + int64_t(m) * ldc + n) = f32x4{v[0], v[1], v[2], v[3]};
        }
      }
    }
    return;
  }
  // ragged N (not a multiple of 4; no serving shape; only the register-staged
  // fallback kernel instantiates it): per element
  if constexpr (!RAGGED) return;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = mb + i * 16 + fr;
    if (m >= M) continue;
    const float sam = (FP8 && sa) ? sa[m] : 1.f;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = nb + j * 16 + fq * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nn = n + r;
        if (nn >= N) break;
        float x = acc[i][j][r];
        if (FP8) x *= (sw ? sw[nn] : 1.f) * sam;
        x = fmaxf(x + (bias ? bias[nn] : 0.f), lo);
        if (sig) x = sigmoidf(x);
        if (cross) x = bf2f(X0[int64_t(m) * ldx + nn]) * x + bf2f(XL[int64_t(m) * ldx + nn]);
        if constexpr (sizeof(OutT) == 2) C[int64_t(m) * ldc + nn] = f2bf(x);
        else C[int64_t(m) * ldc + nn] = x;
      }
    }
  }
}

// DCN-v2 cross epilogue that ALSO emits its output as the next cross layer's
// A operand in OCP MX-fp8: e4m3 values + one E8M0 scale per 32 consecutive
// columns of a row (the K blocks of the consumer's 16x16x128 MFMA). A lane
// holds 4 columns of a row in each of the tile pair (j, j+1) = 32 columns; the
// 4 lanes sharing the row (fq = 0..3, xor-shuffle 16 / 32) reduce the block
// maximum, so no row-wide pass is needed (replaces quant_rows on the cross
// chain). Columns [N, nq) of q are written as zeros (the consumer's K padding).
template <int TM, int TN, typename OutT>
__device__ __forceinline__ void store_cross_mx(const f32x4 (&acc)[TM][TN], int mb, int nb, int fr, int fq, int M, int N,
                                               const float* __restrict__ bias, const float* __restrict__ sa,
                                               const float* __restrict__ sw, OutT* __restrict__ C, int64_t ldc,
                                               const bf16* __restrict__ X0, const bf16* __restrict__ XL, int64_t ldx,
                                               const MxIO& mx) {
  static_assert(TN % 2 == 0, "MX output needs column-tile pairs");
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = mb + i * 16 + fr;
    const bool row_ok = m < M;
    const float sam = (sa && row_ok) ? sa[m] : 1.f;
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      float v[2][4];
      float amax = 0.f;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = nb + (j + h) * 16 + fq * 4;  // N % 32 == 0: all 4 columns in range or none
#pragma unroll
        for (int r = 0; r < 4; ++r) v[h][r] = 0.f;
        if (row_ok && n < N) {
          const bf16x4 x0 = *reinterpret_cast<const bf16x4*>(X0 + int64_t(m) * ldx + n);
          const bf16x4 xl = *reinterpret_cast<const bf16x4*>(XL + int64_t(m) * ldx + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = acc[i][j + h][r] * (sw ? sw[n + r] : 1.f) * sam + (bias ? bias[n + r] : 0.f);
            v[h][r] = bf2f(x0[r]) * x + bf2f(xl[r]);
          }
          if constexpr (sizeof(OutT) == 2) {
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = f2bf(v[h][r]);
            *reinterpret_cast<bf16x4*>(C + int64_t(m) * ldc + n) = o;
          } else {
            *reinterpret_cast<f32x4*>(C + int64_t(m) * ldc + n) = f32x4{v[h][0], v[h][1], v[h][2], v[h][3]};
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) amax = fmaxf(amax, fabsf(v[h][r]));
      }
      // block max over the 4 lanes of this row (lanes fr, fr+16, fr+32, fr+48)
      amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
      // E8M0 exponent: smallest e with amax / 2^e <= 448 (e4m3 max)
      int e = 0;
      if (amax > 0.f) {
        int ex;
        (void)frexpf(amax / 448.f, &ex);  // amax/448 = f * 2^ex, f in [0.5, 1)
        e = ex;
        if (ldexpf(448.f, e - 1) >= amax) e -= 1;
        e = max(-127, min(127, e));
      }
      const float inv = ldexpf(1.f, -e);
      if (!row_ok) continue;
      const int n32 = nb + j * 16;  // first column of the 32-column block
      if (n32 >= mx.nq) continue;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = nb + (j + h) * 16 + fq * 4;
        int w = 0;
        w = __builtin_amdgcn_cvt_pk_fp8_f32(v[h][0] * inv, v[h][1] * inv, w, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(v[h][2] * inv, v[h][3] * inv, w, true);
        *reinterpret_cast<int*>(mx.q + int64_t(m) * mx.ldq + n) = w;
      }
      if (fq == 0) mx.sq[int64_t(m) * mx.ldsq + n32 / 32] = uint8_t(e + 127);
    }
  }
}

template <int BM, int BN, bool FP8, typename OutT>
__global__ void __launch_bounds__(256) gemm_kernel(const uint8_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ W,
                                                   int64_t ldw, const float* __restrict__ bias,
                                                   const float* __restrict__ sa, const float* __restrict__ sw,
                                                   OutT* __restrict__ C, int64_t ldc, const bf16* __restrict__ X0,
                                                   const bf16* __restrict__ XL, int64_t ldx, int M, int N, int K,
                                                   int epi) {
  constexpr int EB = FP8 ? 1 : 2;        // element bytes
  constexpr int BK = 128 / EB;           // elements per K tile
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int CA = BM * 8 / 256;       // 16-B chunks per thread (A)
  constexpr int CB = BN * 8 / 256;
  static_assert(CA >= 1 && CB >= 1, "tile too small");

  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (BM + BN) * 128];
  auto As = [&](int buf) { return smem + buf * ((BM + BN) * 128); };
  auto Bs = [&](int buf) { return smem + buf * ((BM + BN) * 128) + BM * 128; };

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  // consecutive tiles walk M first so one XCD shares W panels
  // Tile order: N-fastest by default, so each XCD's contiguous run of tiles is
  // a few row panels x ALL column panels - the big activation panel is pulled
  // into that XCD's L2 once and reused by every column tile (the weight panel
  // is small). epi bit 4 selects the M-fastest order instead (A/B testing).
  const bool m_fast = (epi & 16) != 0;
  const int tm = m_fast ? tile % tiles_m : tile / tiles_n;
  const int tn = m_fast ? tile / tiles_m : tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int Kb = K * EB;  // row length in bytes

  i32x4 ra[CA], rb[CB];
  auto gload = [&](int kt) {
    const int kb0 = kt * 128;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int id = t + i * 256, r = id >> 3, c = id & 7;
      const int gm = m0 + r, kb = kb0 + c * 16;
      ra[i] = (gm < M && kb < Kb) ? *reinterpret_cast<const i32x4*>(A + gm * lda * EB + kb) : i32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int id = t + i * 256, r = id >> 3, c = id & 7;
      const int gn = n0 + r, kb = kb0 + c * 16;
      rb[i] = (gn < N && kb < Kb) ? *reinterpret_cast<const i32x4*>(W + gn * ldw * EB + kb) : i32x4{0, 0, 0, 0};
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int id = t + i * 256, r = id >> 3, c = id & 7;
      *reinterpret_cast<i32x4*>(As(buf) + swz(r, c)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      const int id = t + i * 256, r = id >> 3, c = id & 7;
      *reinterpret_cast<i32x4*>(Bs(buf) + swz(r, c)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (Kb + 127) / 128;
  gload(0);
  lstore(0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const uint8_t* as = As(cur);
    const uint8_t* bs = Bs(cur);
    if constexpr (!FP8) {
      // bf16: 2 MFMA k-steps of 32 per 64-element tile; lane reads chunk 4*kk + fq.
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(as + swz(wm * WM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * WN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    } else {
      // fp8: one block-scaled 16x16x128 MFMA per output tile covers the whole
      // 128-element K tile (the loader zero-fills past K, so a partial last
      // tile contributes zeros)
      i32x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = mx_frag(as, wm * WM + i * 16 + fr, fq);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = mx_frag(bs, wn * WN + j * 16 + fr, fq);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mx_mfma(bfr[j], af[i], acc[i][j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  store_acc_t<FP8>(acc, m0 + wm * WM, n0 + wn * WN, fr, fq, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, epi);
}

// ---------------------------------------------------------------------------
// LDS-DMA variant (cdna_hip_programming.md §5 "global_load_lds", 2-phase
// structure): tiles go global -> LDS with global_load_lds_dwordx4 (no VGPR
// round trip, no ds_write pass). The LDS image stays lane-linear (one
// wave-instruction = 8 rows x 128 B) and the XOR swizzle moves to the per-lane
// SOURCE chunk (rule 21), so the fragment reads use the same swz() as above.
// Requires K % (128 / elem bytes) == 0; rows past M / N are clamped (their
// results are never stored).
constexpr int kMxMaxKBlocks = 96;  // MX-scaled A: K <= 3072 (the scale panel lives in LDS)

// MXM (fp8 only): bit 0 = MX block scales on A (mx.sab), bit 1 = MX-fp8 output
// (mx.q); separate instantiations, so the plain kernels keep their registers.
template <int BM, int BN, int WM_, int WN_, bool FP8, typename OutT, int MXM = 0>
__device__ __forceinline__ void gemm_glds_body(
    const uint8_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ W, int64_t ldw,
    const float* __restrict__ bias, const float* __restrict__ sa, const float* __restrict__ sw, OutT* __restrict__ C,
    int64_t ldc, const bf16* __restrict__ X0, const bf16* __restrict__ XL, int64_t ldx, int M, int N, int K, int epi,
    const MxIO& mx) {
  constexpr int NW = WM_ * WN_;
  constexpr int EB = FP8 ? 1 : 2;
  constexpr int WTM = BM / WM_, WTN = BN / WN_;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int IA = BM / 8, IB = BN / 8;  // 1-KiB LDS-DMA instructions per tile
  static_assert(IA % NW == 0 && IB % NW == 0, "tile rows must split evenly over waves");
  constexpr int STAGE_BYTES = (BM + BN) * 128;

  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE_BYTES];

  // an MX-fp8 output also covers its zero K-padding columns [N, nq)
  const int tiles_n = (((MXM & 2) ? max(N, mx.nq) : N) + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  // Tile order: N-fastest by default, so each XCD's contiguous run of tiles is
  // a few row panels x ALL column panels - the big activation panel is pulled
  // into that XCD's L2 once and reused by every column tile (the weight panel
  // is small). epi bit 4 selects the M-fastest order instead (A/B testing).
  const bool m_fast = (epi & 16) != 0;
  const int tm = m_fast ? tile % tiles_m : tile / tiles_n;
  const int tn = m_fast ? tile / tiles_m : tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN_, wn = wid % WN_;

  // per-lane source offsets (row within the 8-row group, swizzled chunk)
  const int lr = lane >> 3, ls = lane & 7;
  int64_t a_off[IA / NW], b_off[IB / NW];
#pragma unroll
  for (int j = 0; j < IA / NW; ++j) {
    const int r = 8 * (wid + j * NW) + lr;
    const int gm = min(m0 + r, M - 1);
    a_off[j] = int64_t(gm) * lda * EB + ((ls ^ ((r >> 1) & 7)) << 4);
  }
#pragma unroll
  for (int j = 0; j < IB / NW; ++j) {
    const int r = 8 * (wid + j * NW) + lr;
    const int gn = min(n0 + r, N - 1);
    b_off[j] = int64_t(gn) * ldw * EB + ((ls ^ ((r >> 1) & 7)) << 4);
  }
  auto stage = [&](int buf, int kt) {
    uint8_t* base = smem + buf * STAGE_BYTES;
    const int64_t kb0 = int64_t(kt) * 128;
#pragma unroll
    for (int j = 0; j < IA / NW; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(A + a_off[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + (wid + j * NW) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < IB / NW; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(W + b_off[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + BM * 128 + (wid + j * NW) * 1024),
                                       16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K * EB) / 128;
  const int fr = lane & 15, fq = lane >> 4;
  // MX activation block scales: this lane's row of fragment i, K block 4 kt + fq;
  // prefetched one K tile ahead (the end-of-tile barrier waits for them).
  // MX activation block scales: the block's whole [BM x K/32] scale panel is
  // staged in LDS once (coalesced), laid out [K block][wave row group][fr][i]
  // so a lane's TM scale bytes for one K block are one contiguous LDS word
  // (per-K-tile scattered byte loads from global measured ~1.5x slower).
  // The panel's dword loads are all issued before tile 0's DMA, and their LDS
  // writes land before the barrier that waits for tile 0 (one round trip).
  __shared__ __attribute__((aligned(16))) uint8_t sscale[(MXM & 1) ? kMxMaxKBlocks * BM : 4];
  constexpr int NSW = (MXM & 1) ? (BM * kMxMaxKBlocks / 4 + NW * 64 - 1) / (NW * 64) : 1;
  uint32_t swv[NSW];
  const int KBW = K / 128;  // scale dwords per row
  if constexpr ((MXM & 1) != 0) {
#pragma unroll
    for (int u = 0; u < NSW; ++u) {
      const int idx = threadIdx.x + u * NW * 64;
      if (idx < BM * KBW) {
        const int r = idx / KBW, c = idx - r * KBW;
        const int gm = min(m0 + r, M - 1);
        swv[u] = *reinterpret_cast<const uint32_t*>(mx.sab + int64_t(gm) * mx.ldsab + 4 * c);
      }
    }
  }
  stage(0, 0);
  if constexpr ((MXM & 1) != 0) {
#pragma unroll
    for (int u = 0; u < NSW; ++u) {
      const int idx = threadIdx.x + u * NW * 64;
      if (idx < BM * KBW) {
        const int r = idx / KBW, c = idx - r * KBW;
        const int pos = (r / WTM) * WTM + (r % 16) * TM + (r % WTM) / 16;
#pragma unroll
        for (int t = 0; t < 4; ++t) sscale[(4 * c + t) * BM + pos] = uint8_t(swv[u] >> (8 * t));
      }
    }
  }
  __syncthreads();  // vmcnt(0) + barrier: tile 0 (and the scale panel) landed
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    // this K tile's MX scale word, read BEFORE the next tile's DMA is issued
    // (an LDS read after it makes the compiler wait for the DMA first)
    uint32_t sw4 = 0;
    if constexpr ((MXM & 1) != 0) {
      const uint8_t* sp = sscale + (4 * kt + fq) * BM + wm * WTM + fr * TM;
      if constexpr (TM == 4) sw4 = *reinterpret_cast<const uint32_t*>(sp);
      else if constexpr (TM == 2) sw4 = *reinterpret_cast<const uint16_t*>(sp);
      else sw4 = *sp;
    }
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);  // DMA of the next tile under this tile's MFMAs

    const uint8_t* as = smem + cur * STAGE_BYTES;
    const uint8_t* bs = as + BM * 128;
    if constexpr (!FP8) {
      // Issue every fragment read of the K tile (both 32-deep halves) before
      // the first MFMA, so the second half's LDS latency hides under the
      // first half's MFMAs (the compiler then waits lgkmcnt(N), not 0).
      bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[kk][i] = *reinterpret_cast<const bf16x8*>(as + swz(wm * WTM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[kk][j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * WTN + j * 16 + fr, kk * 4 + fq));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    } else {
      i32x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = mx_frag(as, wm * WTM + i * 16 + fr, fq);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = mx_frag(bs, wn * WTN + j * 16 + fr, fq);
      if constexpr ((MXM & 1) != 0) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int sbi = int((sw4 >> (8 * i)) & 0xffu);
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mx_mfma_sb(bfr[j], af[i], acc[i][j], sbi);
        }
        __builtin_amdgcn_s_setprio(0);
      } else {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mx_mfma(bfr[j], af[i], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();  // next tile landed (vmcnt(0)) and everyone is done reading this one
  }

  if constexpr (FP8 && (MXM & 2) != 0) {
    store_cross_mx(acc, m0 + wm * WTM, n0 + wn * WTN, fr, fq, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, mx);
    return;
  }
  store_acc_t<FP8, false>(acc, m0 + wm * WTM, n0 + wn * WTN, fr, fq, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, epi);
}

#define DTFS_GLDS_ARGS                                                                                              \
  const uint8_t *__restrict__ A, int64_t lda, const uint8_t *__restrict__ W, int64_t ldw,                           \
      const float *__restrict__ bias, const float *__restrict__ sa, const float *__restrict__ sw,                   \
      OutT *__restrict__ C, int64_t ldc, const bf16 *__restrict__ X0, const bf16 *__restrict__ XL, int64_t ldx,     \
      int M, int N, int K, int epi, MxIO mx

template <int BM, int BN, int WM_, int WN_, bool FP8, typename OutT, int MXM>
__global__ void __launch_bounds__(WM_* WN_ * 64) gemm_glds_kernel(DTFS_GLDS_ARGS) {
  gemm_glds_body<BM, BN, WM_, WN_, FP8, OutT, MXM>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi,
                                                   mx);
}

template <int BM, int BN, int WM_, int WN_, bool FP8, int MXM = 0, typename OutT>
static void launch_glds(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                        const float* sw, OutT* C, int64_t ldc, const bf16* X0, const bf16* XL, int64_t ldx, int M,
                        int N, int K, int epi, hipStream_t st, const MxIO& mx = MxIO()) {
  const int Nt = (MXM & 2) ? (N > mx.nq ? N : mx.nq) : N;
  const int grid = ((M + BM - 1) / BM) * ((Nt + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_glds_kernel<BM, BN, WM_, WN_, FP8, OutT, MXM>), dim3(grid), dim3(WM_ * WN_ * 64), 0, st,
                     static_cast<const uint8_t*>(A), lda, static_cast<const uint8_t*>(W), ldw, bias, sa, sw, C, ldc,
                     X0, XL, ldx, M, N, K, epi, mx);
}

// ---------------------------------------------------------------------------
// K4+K6 fused: the last MLP layer and the CTR head in one kernel.
//   h = act(A W^T + b)            [M, N]   (never written to memory)
//   y[m] = out_act(h[m,:] . hw + hbias + extra[m])
// One workgroup owns BM rows x ALL N columns (N <= 256), so the row dot
// product is reduced in-block: lanes sharing a row (xor-shuffle over the 16
// column lanes of a 16x16 tile) then the 4 waves through LDS. Saves the head
// kernel, its launch gap and the [M, N] activation round trip. y may be a
// device pointer or a mapped pinned-host pointer (scores land on the host
// straight from the kernel).
template <int BM, int TN>
__global__ void __launch_bounds__(256) gemm_head_kernel(const uint8_t* __restrict__ A, int64_t lda,
                                                        const uint8_t* __restrict__ W, int64_t ldw,
                                                        const float* __restrict__ bias, int act,
                                                        const float* __restrict__ hw, float hbias,
                                                        const float* __restrict__ extra, int extra_n,
                                                        int64_t extra_ld, int out_act, float* __restrict__ y, int M,
                                                        int N, int K) {
  constexpr int WN_ = 4, NW = 4;
  constexpr int BN = 16 * TN * WN_;
  constexpr int TM = BM / 16;
  constexpr int IA = BM / 8, IB = BN / 8;
  static_assert(IA % NW == 0 && IB % NW == 0, "tile rows must split evenly over waves");
  constexpr int STAGE_BYTES = (BM + BN) * 128;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE_BYTES + NW * BM * 4];
  float* red = reinterpret_cast<float*>(smem + 2 * STAGE_BYTES);

  const int m0 = blockIdx.x * BM;
  const int lane = threadIdx.x & 63;
  const int wn = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane >> 3, ls = lane & 7;
  int64_t a_off[IA / NW], b_off[IB / NW];
#pragma unroll
  for (int j = 0; j < IA / NW; ++j) {
    const int r = 8 * (wn + j * NW) + lr;
    a_off[j] = int64_t(min(m0 + r, M - 1)) * lda * 2 + ((ls ^ ((r >> 1) & 7)) << 4);
  }
#pragma unroll
  for (int j = 0; j < IB / NW; ++j) {
    const int r = 8 * (wn + j * NW) + lr;
    b_off[j] = int64_t(min(r, N - 1)) * ldw * 2 + ((ls ^ ((r >> 1) & 7)) << 4);
  }
  auto stage = [&](int buf, int kt) {
    uint8_t* base = smem + buf * STAGE_BYTES;
    const int64_t kb0 = int64_t(kt) * 128;
#pragma unroll
    for (int j = 0; j < IA / NW; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(A + a_off[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + (wn + j * NW) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < IB / NW; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(W + b_off[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + BM * 128 + (wn + j * NW) * 1024),
                                       16, 0, 0);
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (K * 2) / 128;
  const int fr = lane & 15, fq = lane >> 4;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
    const uint8_t* as = smem + cur * STAGE_BYTES;
    const uint8_t* bs = as + BM * 128;
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TM; ++i) af[kk][i] = *reinterpret_cast<const bf16x8*>(as + swz(i * 16 + fr, kk * 4 + fq));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[kk][j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * 16 * TN + j * 16 + fr, kk * 4 + fq));
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
  // epilogue: per-row partial dot over this wave's columns
  float part[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = wn * 16 * TN + j * 16 + fr;
    const bool ok = n < N;
    const float bn = ok ? bias[n] : 0.f;
    const float wv = ok ? hw[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] + bn;
        if (act == EPI_RELU) v = fmaxf(v, 0.f);
        part[i][r] += v * wv;
      }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = part[i][r];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (fr == 0) red[wn * BM + i * 16 + fq * 4 + r] = v;
    }
  __syncthreads();
  for (int row = threadIdx.x; row < BM; row += blockDim.x) {
    const int m = m0 + row;
    if (m >= M) continue;
    float s = hbias;
    for (int e = 0; extra && e < extra_n; ++e) s += extra[e * extra_ld + m];
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w * BM + row];
    y[m] = out_act == EPI_SIGMOID ? sigmoidf(s) : s;
  }
}

// ---------------------------------------------------------------------------
// 256x256 "8-phase" GEMM (cdna_hip_programming.md §5, "The 256² 8-phase
// template": staggered wave groups + counted vmcnt + raw barriers).
//
// 512 threads = 8 waves; wave (wr = wid>>2, wc = wid&3) owns rows 128wr..+128
// and cols 64wc..+64 (acc[8][4] 16x16 tiles). K tile = 128 bytes per row
// (64 bf16 / 128 fp8); two LDS buffers of 64 KiB (A 256 rows | B 256 rows).
// Each K tile is computed in 4 phases, one C quadrant (4 x 2 tiles) each:
//   p0 (qm0,qn0): ds_read A[qm0] + B[qn0]    p1 (qm0,qn1): ds_read B[qn1]
//   p2 (qm1,qn1): ds_read A[qm1]             p3 (qm1,qn0): ds_read B[qn0]
// and every phase stages one quarter of a later K tile with 2 LDS-DMA
// instructions per thread. Quarters are sliced to match the reads - Aq = the
// qm-th 64 rows of both row groups, Bq = the qn-th 32 columns of every wave's 64
// - so each is last read early in its tile and can be restaged two phases later:
//   p0: Aq1(t+1)   p1: Bq0(t+1)   p2: Aq0(t+2)   p3: Bq1(t+2)
// One counted wait per K tile (p3, before its first barrier) retires t+1's
// quarters and keeps t+2's two in flight, so the DMA never drains in the loop.
// Phase = ds_read + stage | s_barrier | lgkmcnt(0) | 16 MFMA | s_barrier; waves
// 4-7 run one barrier behind waves 0-3, so while one group issues its MFMAs
// the other issues its LDS reads / DMA. Hazard rules (guide, "Read a staged
// buffer one phase AFTER the wait that retires it"; WAR >= 2 phases after the
// last read): quarter X of tile u staged at phase s, first read at phase r:
//   Aq0: s=4u-6 r=4u   Bq1: s=4u-5 r=4u+1   Aq1: s=4u-4 r=4u+2   Bq0: s=4u-3 r=4u
// all retired by the wait at phase 4u-1 (<= r-1); restaged >= 2 phases after
// their last reads (Aq0 p0, Bq1 p1, Aq1 p2, Bq0 p3 of tile u-2 / u-1).
// Diagnostic build only (bench_native/g8ph_stamps.hip defines it): lane 0 of
// each wave records s_memrealtime (100 MHz) at kernel entry, after the
// prologue, after the main loop and after the epilogue, into a buffer no
// other code reads. Never defined in the extension build.
#ifdef DTFS_8PH_STAMPS
__device__ unsigned long long g_8ph_stamps[4096][8][4];
#define DTFS_STAMP(k)                                                                        \
  do {                                                                                       \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                          \
    __builtin_amdgcn_s_waitcnt(0xC07F);                                                      \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_8ph_stamps[blockIdx.x][threadIdx.x >> 6][k] = t_; \
  } while (0)
#else
#define DTFS_STAMP(k) \
  do {                \
  } while (0)
#endif

// Diagnostic build only (tools/native/gg_stamps.hip defines it): per-phase
// s_memtime stamps of gemm_gather_kernel for ONE K tile in the middle of the
// loop, kept in registers and written by lane 0 after the epilogue (a store
// inside the loop would shift the counted vmcnt waits), plus entry / prologue /
// loop / epilogue. Never defined in the extension build.
#ifdef DTFS_GG_STAMPS
__device__ unsigned long long g_gg_stamps[4096][8][16];
#define GG_T(k)                                             \
  do {                                                      \
    if (t == gg_t) gg_s[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#define GG_AT(k)                                   \
  do {                                             \
    gg_s[k] = __builtin_amdgcn_s_memtime();        \
  } while (0)
#else
#define GG_T(k) \
  do {          \
  } while (0)
#define GG_AT(k) \
  do {           \
  } while (0)
#endif

// DCN-v2 cross layer epilogue of the 256x256 8-phase tile, staged through LDS
// (XSTAGE): the fused cross epilogue in registers (store_acc_t, EPI_CROSS)
// loads x0 / xl as 8-byte pieces of 16 rows per fragment, one latency-bound
// round trip per column tile with no MFMA work left to hide it (215.6 vs
// 124.7 us plain at 16384 x 2752 x 2816), which is why the split form (plain
// GEMM + an HBM-bound combine pass over y, x0, xl) won in round 2. Here the
// tile's y = bf16(acc * sa * sw + b) - the split form's y, bit for bit - goes
// to LDS (the K loop's buffers are dead; 520-byte rows: the 16 rows of a
// lane group's 8-byte writes land on 32 distinct banks), then every wave
// streams whole rows: 32 lanes x 16 bytes = one 256-column row segment, x0 / xl
// read fully coalesced with 4 rows in flight per lane, z = bf16(x0 * y + xl)
// written back as 16-byte vectors and / or dotted with head_w into one
// partial logit per (column tile, row): dot[tn * ldd + m]. No y round trip
// through HBM and no separate combine pass.
constexpr int kXsLdy = 520;  // staged row pitch (bytes): 256 bf16 + 8
constexpr int kXsBytes = 256 * kXsLdy;
// 32-lane (half-wave) sum with the result in every lane: DPP within each
// 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror), one
// ds_bpermute across the two rows
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float sum32(float v) {
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v + __shfl_xor(v, 16, 64);
}
// The cross GEMM's extra operands (one struct: the 8-phase kernel's argument
// list stays the dense GEMM's otherwise).
struct XsArgs {
  const float* hw = nullptr;  // head weights [N]: per-tile partial logits ...
  float* dot = nullptr;       // ... dot[tn * ldd + m]
  int64_t ldd = 0;
};

template <bool FP8>
__device__ __forceinline__ void cross_staged_epilogue(const f32x4 (&acc)[8][4], uint8_t* __restrict__ ys, int m0,
                                                      int n0, int tn, int wr, int wc, int wid, int lane, int M, int N,
                                                      const float* __restrict__ bias, const float* __restrict__ sa,
                                                      const float* __restrict__ sw, bf16* __restrict__ Z,
                                                      int64_t ldz, const bf16* __restrict__ X0,
                                                      const bf16* __restrict__ XL, int64_t ldx, const XsArgs& xs) {
  const int fr = lane & 15, fq = lane >> 4;
  __syncthreads();  // both wave groups are past their last K-loop LDS read
  // scale / bias vectors and, below, the x0 / xl rows are each loaded in one
  // round trip (a latency-bound epilogue, one tile per CU and nothing else
  // to run: tools/native/g8ph_stamps)
  float sam[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sam[i] = (FP8 && sa) ? sa[min(m0 + 128 * wr + 16 * i + fr, M - 1)] : 1.f;
  f32x4 b4v[4], s4v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nc = min(n0 + 64 * wc + 16 * j + 4 * fq, N - 4);
    b4v[j] = bias ? *reinterpret_cast<const f32x4*>(bias + nc) : f32x4{0.f, 0.f, 0.f, 0.f};
    s4v[j] = (FP8 && sw) ? *reinterpret_cast<const f32x4*>(sw + nc) : f32x4{1.f, 1.f, 1.f, 1.f};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 64 * wc + 16 * j + 4 * fq;  // tile column of this lane's 4 values
    const f32x4 b4 = b4v[j];
    const f32x4 s4 = s4v[j];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r];
        if constexpr (FP8) x *= s4[r] * sam[i];
        o[r] = f2bf(x + b4[r]);
      }
      *reinterpret_cast<bf16x4*>(ys + (128 * wr + 16 * i + fr) * kXsLdy + c * 2) = o;
    }
  }
  __syncthreads();
  // rows: wave wid owns tile rows 32 wid .. +32, two per pass (lanes 0-31 / 32-63)
  const int col = (lane & 31) * 8;
  const int n = n0 + col;
  const bool col_ok = n < N;  // N % 8 == 0: a lane's 8 columns exist together
  const int nr = min(n, N - 8);
  const bool same = XL == X0;
  float w8[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) w8[e] = 0.f;
  if (xs.hw && col_ok) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(xs.hw + n);
    const f32x4 b = *reinterpret_cast<const f32x4*>(xs.hw + n + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) w8[e] = a[e], w8[e + 4] = b[e];
  }
  constexpr int P = 16;  // rows in flight per lane: all of them (the accumulators are dead by now)
#pragma unroll 1
  for (int p0 = 0; p0 < 16; p0 += P) {
    bf16x8 x0v[P], xlv[P];
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int64_t m = min(m0 + 32 * wid + 2 * (p0 + u) + (lane >> 5), M - 1);
      x0v[u] = *reinterpret_cast<const bf16x8*>(X0 + m * ldx + nr);
      if (!same) xlv[u] = *reinterpret_cast<const bf16x8*>(XL + m * ldx + nr);
    }
#pragma unroll
    for (int u = 0; u < P; ++u) {
      const int row = 32 * wid + 2 * (p0 + u) + (lane >> 5);
      const int m = m0 + row;
      const bf16x8 y8 = *reinterpret_cast<const bf16x8*>(ys + row * kXsLdy + col * 2);
      const bf16x8 l8 = same ? x0v[u] : xlv[u];
      bf16x8 z8;
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        z8[e] = f2bf(bf2f(x0v[u][e]) * bf2f(y8[e]) + bf2f(l8[e]));
        d += bf2f(z8[e]) * w8[e];
      }
      if (Z && col_ok && m < M) *reinterpret_cast<bf16x8*>(Z + int64_t(m) * ldz + n) = z8;
      if (xs.dot) {
        d = sum32(d);
        if ((lane & 31) == 0 && m < M) xs.dot[int64_t(tn) * xs.ldd + m] = d;
      }
    }
  }
}

// Plain (bias / ReLU / sigmoid) epilogue of a 256x256 tile, staged through
// LDS like the cross epilogue above. In registers each store instruction of
// the transposed layout writes 32 bytes into each of 16 rows (16 partial
// lines per instruction, 32 instructions per wave): tools/native/g8ph_stamps
// measured 6.8 us for one tile's epilogue with nothing else running (the
// staged cross epilogue, which also reads x0 / xl, took 5.6). Staged, a store
// instruction writes two 512-byte row segments (8 whole lines), half as many
// instructions. bf16 output, N % 8 == 0 and ldc % 8 == 0 (16-byte rows).
template <bool FP8>
__device__ __forceinline__ void plain_staged_epilogue(const f32x4 (&acc)[8][4], uint8_t* __restrict__ ys, int m0,
                                                      int n0, int wr, int wc, int wid, int lane, int M, int N,
                                                      const float* __restrict__ bias, const float* __restrict__ sa,
                                                      const float* __restrict__ sw, bf16* __restrict__ C, int64_t ldc,
                                                      int epi) {
  const int fr = lane & 15, fq = lane >> 4;
  const int e = epi & 15;
  const bool sig = e == EPI_SIGMOID;
  const float lo = e == EPI_RELU ? 0.f : -__builtin_huge_valf();
  __syncthreads();  // both wave groups are past their last K-loop LDS read
  float sam[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sam[i] = (FP8 && sa) ? sa[min(m0 + 128 * wr + 16 * i + fr, M - 1)] : 1.f;
  f32x4 b4v[4], s4v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int nc = min(n0 + 64 * wc + 16 * j + 4 * fq, N - 4);
    b4v[j] = bias ? *reinterpret_cast<const f32x4*>(bias + nc) : f32x4{0.f, 0.f, 0.f, 0.f};
    s4v[j] = (FP8 && sw) ? *reinterpret_cast<const f32x4*>(sw + nc) : f32x4{1.f, 1.f, 1.f, 1.f};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 64 * wc + 16 * j + 4 * fq;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r];
        if constexpr (FP8) x *= s4v[j][r] * sam[i];
        v[r] = fmaxf(x + b4v[j][r], lo);
      }
      if (sig) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = sigmoidf(v[r]);
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
      *reinterpret_cast<bf16x4*>(ys + (128 * wr + 16 * i + fr) * kXsLdy + c * 2) = o;
    }
  }
  __syncthreads();
  const int col = (lane & 31) * 8;
  const int n = n0 + col;
  if (n >= N) return;
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const int row = 32 * wid + 2 * p + (lane >> 5);
    const int m = m0 + row;
    if (m < M)
      *reinterpret_cast<bf16x8*>(C + int64_t(m) * ldc + n) = *reinterpret_cast<const bf16x8*>(ys + row * kXsLdy + col * 2);
  }
}

template <bool FP8, typename OutT, bool PRE = false, bool XSTAGE = false>
__global__ void __launch_bounds__(512) gemm_8ph_kernel(
    const uint8_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ W, int64_t ldw,
    const float* __restrict__ bias, const float* __restrict__ sa, const float* __restrict__ sw, OutT* __restrict__ C,
    int64_t ldc, const bf16* __restrict__ X0, const bf16* __restrict__ XL, int64_t ldx, int M, int N, int K, int epi,
    const XsArgs xs) {
  constexpr int BM = 256, BN = 256;
  constexpr int EB = FP8 ? 1 : 2;
  constexpr int BUF = (BM + BN) * 128;  // 64 KiB
  constexpr int KLOOP = 2 * BUF;
  constexpr int SMEM = kXsBytes > KLOOP ? kXsBytes : KLOOP;  // the staged epilogues reuse the K-loop buffers
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  DTFS_STAMP(0);

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  // N-fastest inside each XCD's contiguous share (a grouped M-fastest order,
  // gm row tiles x 32 / gm column tiles in flight, measured within 0.7 %:
  // profiles/r06_dcn_cross_tile_order.md)
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int lr = lane >> 3, ls = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;

  const int nk = (K * EB) / 128;
  // staging geometry: quarter q of A / B = 16 groups of 8 contiguous LDS rows;
  // this wave stages groups wid and wid + 8 of every quarter
  auto a_row = [&](int qm, int g) { return (g < 8 ? 0 : 128) + 64 * qm + 8 * (g & 7); };
  auto b_row = [&](int qn, int g) { return 64 * (g >> 2) + 32 * qn + 8 * (g & 3); };
  int64_t a_src[2][2], b_src[2][2];  // [quarter][j]
  int a_dst[2][2], b_dst[2][2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int g = wid + 8 * j;
      const int ra = a_row(q, g), rb = b_row(q, g);
      const int r_a = ra + lr, r_b = rb + lr;  // this lane's LDS row
      a_src[q][j] = int64_t(min(m0 + r_a, M - 1)) * lda * EB + ((ls ^ ((r_a >> 1) & 7)) << 4);
      b_src[q][j] = int64_t(min(n0 + r_b, N - 1)) * ldw * EB + ((ls ^ ((r_b >> 1) & 7)) << 4);
      a_dst[q][j] = ra * 128;
      b_dst[q][j] = BM * 128 + rb * 128;
    }
  // tiles past the end (the loop stages unconditionally, see below) re-load
  // the last tile into the buffer nobody reads any more
  auto stage_a = [&](int q, int kt) {
    uint8_t* base = smem + (kt & 1) * BUF;
    const int64_t kb = int64_t(min(kt, nk - 1)) * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(A + a_src[q][j] + kb),
                                       (__attribute__((address_space(3))) void*)(base + a_dst[q][j]), 16, 0, 0);
  };
  auto stage_b = [&](int q, int kt) {
    uint8_t* base = smem + (kt & 1) * BUF;
    const int64_t kb = int64_t(min(kt, nk - 1)) * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(W + b_src[q][j] + kb),
                                       (__attribute__((address_space(3))) void*)(base + b_dst[q][j]), 16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: tile 0 whole + tile 1's Aq0, Bq0 (staged at phases -2, -1 of the
  // steady-state schedule below)
  stage_a(0, 0);
  stage_b(0, 0);
  stage_b(1, 0);
  stage_a(1, 0);
  if (nk > 1) {
    stage_a(0, 1);
    stage_b(0, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
  asm volatile("" ::: "memory");
  DTFS_STAMP(1);

  // fragments (bf16: [kk][tile] 8 x bf16, fp8: [tile] 32 x e4m3); both B
  // column halves stay in registers for the whole K tile (no B re-read)
  // PRE: two A fragment sets - [0] holds A[qm0], [1] A[qm1] - and A[qm0] of
  // the NEXT K tile is read in phase 3 (which reads nothing otherwise), so the
  // LDS reads per phase are 4 / 4 / 8 / 8 instead of 12 / 4 / 8 / 0. Next
  // tile's Aq0 was staged 5 phases before p3 and retired by p2's wait (RAW
  // s + 5 holds); its restage (tile t + 3) is 3 phases after this read.
  constexpr int NA = PRE ? 2 : 1;
  bf16x8 fa[NA][2][4], fb[2][2][2];
  i32x8 xa[NA][4], xb[2][2];
  auto read_a_into = [&](const uint8_t* buf, int qm, int set) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 128 * wr + 64 * qm + 16 * i + fr;
      if constexpr (FP8) {
        xa[set][i] = mx_frag(buf, row, fq);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          fa[set][kk][i] = *reinterpret_cast<const bf16x8*>(buf + swz(row, kk * 4 + fq));
      }
    }
  };
  auto read_a = [&](const uint8_t* buf, int qm) { read_a_into(buf, qm, PRE ? qm : 0); };
  auto read_b = [&](const uint8_t* buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 64 * wc + 32 * qn + 16 * j + fr;
      if constexpr (FP8) {
        xb[qn][j] = mx_frag(buf + BM * 128, row, fq);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          fb[qn][kk][j] = *reinterpret_cast<const bf16x8*>(buf + BM * 128 + swz(row, kk * 4 + fq));
      }
    }
  };
  // one quadrant: 4 x 2 output tiles (transposed MFMA: D = W . A^T, see store_acc_t)
  // sched_barrier(0) pins the quadrant's MFMAs inside their phase: without it
  // the scheduler sinks every (register-only) scaled fp8 MFMA of the K tile
  // past the phase barriers to the end of the iteration (seen in the gfx950
  // ISA), which serialises the two wave groups instead of overlapping them
  auto mma = [&](int qm, int qn) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
    const int set = PRE ? qm : 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4& c = acc[4 * qm + i][2 * qn + j];
        if constexpr (FP8) {
          c = mx_mfma(xb[qn][j], xa[set][i], c);
        } else {
#pragma unroll
          for (int kk = 0; kk < 2; ++kk)
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[qn][kk][j], fa[set][kk][i], c, 0, 0, 0);
        }
      }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // Phase = reads | stage one quarter | counted wait | barrier | MFMAs | barrier
  //   p0: read A[qm0] B[qn0], stage Bq1(t+1)      p1: read B[qn1], stage Aq1(t+1)
  //   p2: read A[qm1],        stage Aq0(t+2)      p3: (no reads), stage Bq0(t+2)
  // WAR: each quarter is restaged >= 2 phases after its last read (Aq0, Bq0 at
  // p0; Bq1 p1; Aq1 p2). RAW: a quarter staged at phase s is retired by the
  // wait of phase s+4 (vmcnt(8): the 4 most recent quarters, 2 DMA
  // instructions each, stay in flight) and first read at phase >= s+5.
  // The loop body is branch-free: the stages of tiles nk and nk+1 are issued
  // too (re-loading the last tile, into buffers no later phase reads; same WAR
  // spacing as every other stage), so every wait is the same vmcnt(8) and the
  // whole K tile is ONE basic block. With per-phase branches the scheduler
  // sank every scaled fp8 MFMA of the tile past the phase barriers into the
  // loop latch (gfx950 ISA), serialising the two wave groups;
  // sched_barrier(0) in mma() then pins each quadrant inside its phase.
  auto wait_dma = [] { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); };
  if constexpr (PRE) read_a(smem, 0);  // tile 0's A[qm0] (landed: the prologue's wait + barrier)
  for (int t = 0; t < nk; ++t) {
    const uint8_t* buf = smem + (t & 1) * BUF;
    // p0
    if constexpr (!PRE) read_a(buf, 0);
    read_b(buf, 0);
    stage_b(1, t + 1);
    wait_dma();
    barrier();
    mma(0, 0);
    barrier();
    // p1
    read_b(buf, 1);
    stage_a(1, t + 1);
    wait_dma();
    barrier();
    mma(0, 1);
    barrier();
    // p2
    read_a(buf, 1);
    stage_a(0, t + 2);
    wait_dma();
    barrier();
    mma(1, 1);
    barrier();
    // p3
    if constexpr (PRE) read_a(smem + ((t + 1) & 1) * BUF, 0);  // next tile's A[qm0] (dead data after the last)
    stage_b(0, t + 2);
    wait_dma();
    barrier();
    mma(1, 0);
    barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing stages land before the waves exit
  if (wr == 0) __builtin_amdgcn_s_barrier();  // match the staggered group's barrier count
  DTFS_STAMP(2);

  if constexpr (XSTAGE) {
    static_assert(sizeof(OutT) == 2, "the staged cross epilogue writes bf16 z");
    cross_staged_epilogue<FP8>(acc, smem, m0, n0, tn, wr, wc, wid, lane, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, xs);
  } else if (sizeof(OutT) == 2 && (epi & 15) != EPI_CROSS && ((N | int(ldc)) & 7) == 0) {
    plain_staged_epilogue<FP8>(acc, smem, m0, n0, wr, wc, wid, lane, M, N, bias, sa, sw,
                               reinterpret_cast<bf16*>(C), ldc, epi);
  } else {
    store_acc_t<FP8, false>(acc, m0 + 128 * wr, n0 + 64 * wc, fr, fq, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, epi);
  }
  DTFS_STAMP(3);
}

template <bool FP8, typename OutT, bool PRE = false>
static void launch_8ph(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                       const float* sw, OutT* C, int64_t ldc, const bf16* X0, const bf16* XL, int64_t ldx, int M,
                       int N, int K, int epi, hipStream_t st) {
  const int grid = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL((gemm_8ph_kernel<FP8, OutT, PRE>), dim3(grid), dim3(512), 0, st, static_cast<const uint8_t*>(A), lda,
                     static_cast<const uint8_t*>(W), ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, XsArgs());
}

// ---------------------------------------------------------------------------
// K1 fused into K4: the first MLP layer of DeepFM / WDL straight from the
// embedding table (the north star's "LDS-staged sparse gather"):
//   C[m, n] = act( sum_f bf16(w[m,f] * T[row(m,f)]) . W[n, 64f .. 64f+63] + b[n] )
// on the 8-phase schedule of gemm_8ph_kernel (plain form). K tile f is field f:
// its A tile is the 128-byte table row of each of the block's 256 candidates,
// staged by the same LDS-DMA instructions as the dense kernel but from
// table + row * 128 per lane. The rows and weights of a K tile come from
// embed_resolve_kernel's field-major rows_t / wts_t [F][Mp] through an 8-slot
// LDS ring: ONE LDS-DMA per wave per K tile, issued in phase 1 four tiles
// ahead (in phase 0, three ahead, it crowded the phase that already issues 4
// quarter DMAs: 104.4 vs 107.9 us at 16384 rows). A stage's rows are read from
// the ring a phase before it (mma()'s lgkmcnt(0) covers the read).
//
// The weights are applied ONCE per element, in LDS: x = bf16(w * e) (the
// unfused gather's rounding, bit for bit) by a scale pass over each landed A
// quarter - every thread rescales two 16-byte chunks in place - in a phase
// that has no other use for that quarter. Scaling the MFMA fragments instead
// costs each of the 4 column waves the same work again (measured: +48 us of
// VALU on the 146 us kernel at 16384 rows); the pass adds 2 x 16 KB of LDS
// traffic per K tile and ~40 VALU per wave, issued between the MFMAs. For the
// spare phase Aq1 is staged one phase earlier than in the dense kernel:
//   p0: stage Bq1(t+1) Aq1(t+1)   p1: scale Aq1(t), ring(t+4)
//   p2: stage Aq0(t+2)             p3: scale Aq0(t+1), stage Bq0(t+2)
// 4 + 1 + 2 + 2 = 9 DMA instructions per 4 phases, so the counted wait
// vmcnt(9) retires every DMA issued 4 phases earlier (quarters, ring alike):
// ring(u) lands by phase 1 of tile u-3, one phase before its first read
// (phase 1 of tile u-2 reads the rows for Aq0(u)).
// Each quarter is loaded for scaling one phase after the wait that retires it
// (the read segment, so the other group has passed that wait too) and read by
// the MFMA phase after that: a group scales only the rows it reads, so its
// own lgkmcnt(0) + barrier at the end of the scaling phase order the writes. WAR:
// Aq1(t+1) overwrites buffer (t+1)&1 two phases after Aq1(t-1)'s last read
// (p2 of tile t-1); the other quarters as in the dense kernel.
//
// FM (DeepFM) rides on the scale pass, which holds e and w in fp32: column
// tile tn < 4 accumulates, for quarter tn >> 1 and row half tn & 1 of each
// group, each thread's 8 dims of one candidate (sum_f v, sum_f v^2, v = e * w);
// 8 lanes finish the row, so every candidate's second-order term
//   fm_part[Mp + m] = 0.5 * (sum_d (sum_f v_fd)^2 - sum_{f,d} v_fd^2)
// comes from exactly one tile, and the head adds it to part0 (bias + first
// order, from the resolve kernel): no second pass over the table. DCN (EXTRA
// 2) takes the same rows' L + 1 cross dot products instead and writes the
// cross logit there.
// EXTRA: what rides on the scale pass - 0 nothing (WDL), 1 the FM
// second-order term (DeepFM), 2 the DCN v1 cross network (K3): the L + 1 dot
// products of x0 with the folded cross weights (embedding.hip "K3 in the
// gather"), whose K-tile slices travel through a third ring.
template <typename OutT, int EXTRA>
__global__ void __launch_bounds__(512) gemm_gather_kernel(const uint8_t* __restrict__ table, int Vm1,
                                                          const int32_t* __restrict__ rows_t,
                                                          const float* __restrict__ wts_t, int64_t Mp,
                                                          const uint8_t* __restrict__ W, const float* __restrict__ bias,
                                                          OutT* __restrict__ C, int64_t ldc, float* __restrict__ fm_part,
                                                          const float* __restrict__ cross_w,
                                                          const float* __restrict__ cross_c, int cross_n, int M, int N,
                                                          int F, int epi) {
  constexpr int BM = 256, BN = 256;
  constexpr int BUF = (BM + BN) * 128;  // 64 KiB
  constexpr int RING = 8;
  constexpr int XMAX = 4;  // cross weight rows per K tile (L + 1 <= 4)
#ifdef DTFS_GG_STAMPS
  unsigned long long gg_s[16] = {};
  const int gg_t = F / 2;
  gg_s[13] = __builtin_amdgcn_s_memrealtime();
#endif
  GG_AT(0);
  // one LDS object (A/B double buffer | ring rows | ring weights | ring cross
  // weights): separate __shared__ arrays made the compiler put vmcnt(0) in
  // front of the A-tile reads (LDS-DMA alias tracking), draining the DMA
  // pipeline twice a K tile
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF + 3 * RING * BM * 4];
  int32_t(*s_rows)[BM] = reinterpret_cast<int32_t(*)[BM]>(smem + 2 * BUF);
  float(*s_wts)[BM] = reinterpret_cast<float(*)[BM]>(smem + 2 * BUF + RING * BM * 4);
  float(*s_xw)[XMAX][64] = reinterpret_cast<float(*)[XMAX][64]>(smem + 2 * BUF + 2 * RING * BM * 4);

  const int tiles_n = N / BN, tiles_m = int(Mp / BM);
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int lr = lane >> 3, ls = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = F;
  const int64_t ldw = int64_t(F) * 64;

  auto a_row = [&](int qm, int g) { return (g < 8 ? 0 : 128) + 64 * qm + 8 * (g & 7); };
  auto b_row = [&](int qn, int g) { return 64 * (g >> 2) + 32 * qn + 8 * (g & 3); };
  // Every staged row r = (multiple of 8) + lr has swizzle (r >> 1) & 7 =
  // 4 (wid & 1) | (lr >> 1) (a_row / b_row of group wid + 8j), so one per-lane
  // chunk offset serves every A and B stage; the row parts are wave-uniform
  // (kept in SGPRs: the kernel sits near the 256-VGPR limit of 2 waves / SIMD).
  const int coff = (ls ^ ((4 * (wid & 1)) | (lr >> 1))) << 4;
  const int b_lane = lr * int(ldw) * 2 + coff;  // N * K * 2 < 2^31 (launcher)
  // ring: ONE 16-byte-per-lane LDS-DMA per wave per K tile (so every wave's
  // counted waits stay identical): wave w fetches kind w % 3 - tile u's 256
  // rows (1 KiB), their weights, or the cross weights' 64-column slices (lane
  // l: row l >> 4, columns 4 (l & 15) ..; a dummy re-fetch of the rows
  // without a cross network) - kinds fetched by two or three waves write the
  // same bytes twice
  const int rk = wid % 3;
  auto stage_ring = [&](int u) {
    const int uc = min(u, nk - 1), slot = u & (RING - 1);
    const void* g;
    void* l;
    if (rk == 2 && EXTRA == 2) {
      const int xr = min(lane >> 4, cross_n - 1);
      g = cross_w + int64_t(xr) * F * 64 + uc * 64 + (lane & 15) * 4;
      l = &s_xw[slot][0][0];
    } else {
      const int64_t src = int64_t(uc) * Mp + m0 + lane * 4;
      g = rk == 1 ? static_cast<const void*>(wts_t + src) : static_cast<const void*>(rows_t + src);
      l = rk == 1 ? static_cast<void*>(&s_wts[slot][0])
                  : (rk == 0 ? static_cast<void*>(&s_rows[slot][0]) : static_cast<void*>(&s_xw[slot][0][0]));
    }
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(g),
                                     (__attribute__((address_space(3))) void*)(l), 16, 0, 0);
  };
  int ida[2];  // table rows of the next A stage
  auto read_rows = [&](int q, int kt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) ida[j] = s_rows[kt & (RING - 1)][a_row(q, wid + 8 * j) + lr];
  };
  auto stage_a = [&](int q, int kt) {
    uint8_t* base = smem + (kt & 1) * BUF;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = min(max(ida[j], 0), Vm1);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(table + int64_t(r) * 128 + coff),
                                       (__attribute__((address_space(3))) void*)(base + a_row(q, wid + 8 * j) * 128),
                                       16, 0, 0);
    }
  };
  auto stage_b = [&](int q, int kt) {
    uint8_t* base = smem + (kt & 1) * BUF;
    const int64_t kb = int64_t(min(kt, nk - 1)) * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int rb = b_row(q, wid + 8 * j);  // n0 + rb + lr < N: N % 256 == 0
      const uint8_t* src = W + (int64_t(n0 + rb) * ldw * 2 + kb) + uint32_t(b_lane);
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src),
                                       (__attribute__((address_space(3))) void*)(base + BM * 128 + rb * 128), 16, 0, 0);
    }
  };

  // scale pass, group-local: wave group wr only ever reads A rows 128 wr ..
  // 128 wr + 127, so it scales exactly those rows of a quarter (64 q + rr and
  // 64 q + rr + 32 within the group, chunk ch; a wave covers 8 whole rows,
  // 1 KiB, conflict-free) and only its own barriers order the writes before its
  // reads. The chunks are loaded in a phase's read segment (retired by then) and
  // rescaled + written back in its MFMA segment, between the MFMAs.
  const int sp_rr = (threadIdx.x & 255) >> 3, sp_ch = threadIdx.x & 7;
  // the logical 8-dim chunk this thread always holds (rows 64 q + rr + 32 h all
  // share the swizzle (rr >> 1) & 7)
  const int sp_dim = 8 * (sp_ch ^ ((sp_rr >> 1) & 7));
  const bool fm_on = EXTRA != 0 && fm_part != nullptr && tn < 4;
  const int fm_q = tn >> 1, fm_h = tn & 1;
  constexpr int NFS = EXTRA == 1 ? 8 : (EXTRA == 2 ? XMAX : 1);
  float fs[NFS], fsq = 0.f;  // FM: per-dim sums + sum of squares; cross: the dot products
#pragma unroll
  for (int j = 0; j < NFS; ++j) fs[j] = 0.f;
  i32x4 su[2];
  float sw[2];
  auto scale_row = [&](int q, int h) { return 128 * wr + 64 * q + sp_rr + 32 * h; };
  auto scale_load = [&](const uint8_t* buf, int q, int u) {
#ifdef DTFS_GG_NO_SCALE  // diagnostic build only: timing without the scale pass (wrong results)
    return;
#endif
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = scale_row(q, h);
      su[h] = *reinterpret_cast<const i32x4*>(buf + r * 128 + sp_ch * 16);
      sw[h] = s_wts[u & (RING - 1)][r];
    }
  };
  auto scale_store = [&](uint8_t* buf, int q, int u) {
#ifdef DTFS_GG_NO_SCALE
    return;
#endif
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      i32x4 o;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        int r;
        asm("v_cvt_pk_bf16_f32 %0, %1, %2"
            : "=v"(r)
            : "v"(__uint_as_float(uint32_t(su[h][p]) << 16) * sw[h]),
              "v"(__uint_as_float(uint32_t(su[h][p]) & 0xffff0000u) * sw[h]));
        o[p] = r;
      }
      *reinterpret_cast<i32x4*>(buf + scale_row(q, h) * 128 + sp_ch * 16) = o;
    }
    // FM: tile tn (< 4) takes quarter tn >> 1, row half tn & 1 of every group,
    // so each candidate's term comes from one tile (one wave-uniform branch per
    // pass; u == nk is the loop's trailing re-staged, dead tile)
    if (fm_on && q == fm_q && u < nk) {
      const i32x4 uf = fm_h ? su[1] : su[0];
      const float wf = fm_h ? sw[1] : sw[0];
      float v[8];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        v[2 * p] = __uint_as_float(uint32_t(uf[p]) << 16) * wf;
        v[2 * p + 1] = __uint_as_float(uint32_t(uf[p]) & 0xffff0000u) * wf;
      }
      if constexpr (EXTRA == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          fs[j] += v[j];
          fsq += v[j] * v[j];
        }
      } else if constexpr (EXTRA == 2) {
#pragma unroll
        for (int l = 0; l < XMAX; ++l) {
          const f32x4 c0 = *reinterpret_cast<const f32x4*>(&s_xw[u & (RING - 1)][l][sp_dim]);
          const f32x4 c1 = *reinterpret_cast<const f32x4*>(&s_xw[u & (RING - 1)][l][sp_dim + 4]);
          fs[l] += v[0] * c0[0] + v[1] * c0[1] + v[2] * c0[2] + v[3] * c0[3] + v[4] * c1[0] + v[5] * c1[1] +
                   v[6] * c1[2] + v[7] * c1[3];
        }
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: the ring for tiles 0-2, tile 0 whole + tile 1's Aq0 / Bq0, tile
  // 0's Aq0 scaled by everyone, then the stagger
  stage_ring(0);
  stage_ring(1);
  stage_ring(2);
  stage_ring(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  read_rows(0, 0);
  stage_a(0, 0);
  stage_b(0, 0);
  stage_b(1, 0);
  read_rows(1, 0);
  stage_a(1, 0);
  read_rows(0, 1);
  stage_a(0, 1);
  stage_b(0, 1);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  __syncthreads();
  scale_load(smem, 0, 0);  // tile 0's Aq0 (Aq1(0) is scaled by the loop's first phase 1)
  scale_store(smem, 0, 0);
  read_rows(1, 1);  // p0(0) stages Aq1(1)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 one barrier behind
  asm volatile("" ::: "memory");
  GG_AT(1);

  bf16x8 fa[2][4], fb[2][2][2];
  auto read_a = [&](const uint8_t* buf, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 128 * wr + 64 * qm + 16 * i + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[kk][i] = *reinterpret_cast<const bf16x8*>(buf + swz(row, kk * 4 + fq));
    }
  };
  auto read_b = [&](const uint8_t* buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = 64 * wc + 32 * qn + 16 * j + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        fb[qn][kk][j] = *reinterpret_cast<const bf16x8*>(buf + BM * 128 + swz(row, kk * 4 + fq));
    }
  };
  // one quadrant's 16 MFMAs; sbuf: also the scale pass of (sq, su) loaded in
  // this phase's read segment, its VALU and stores issued between the MFMAs
  auto mma = [&](int qm, int qn, bool scale = false, uint8_t* sbuf = nullptr, int sq = 0, int su_ = 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        f32x4& c = acc[4 * qm + i][2 * qn + j];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[qn][kk][j], fa[kk][i], c, 0, 0, 0);
      }
    if (scale) {  // a literal at every call: folded, one basic block with the MFMAs
      scale_store(sbuf, sq, su_);
      // interleave: the scale VALU issues while the MFMAs occupy the matrix pipe
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 3 VALU
      }
      __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);    // the 2 LDS stores
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [] {
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto wait_dma = [] { asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); };
  auto wait_lds = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
  for (int t = 0; t < nk; ++t) {
    uint8_t* buf = smem + (t & 1) * BUF;
    uint8_t* nbuf = smem + ((t + 1) & 1) * BUF;
    // p0: A[qm0] B[qn0]; stage Bq1(t+1), Aq1(t+1) (rows read in p3)
    GG_T(2);
    read_a(buf, 0);
    read_b(buf, 0);
    stage_b(1, t + 1);
    stage_a(1, t + 1);
    wait_dma();
    barrier();
    GG_T(3);
    mma(0, 0);
    barrier();
    // p1: B[qn1]; scale Aq1(t) (load here, rescale + store between the MFMAs); rows for p2's stage;
    // the ring for tile t+4
    GG_T(4);
    read_b(buf, 1);
    scale_load(buf, 1, t);
    read_rows(0, t + 2);
    stage_ring(t + 4);
    wait_dma();
    barrier();
    GG_T(5);
    mma(0, 1, true, buf, 1, t);
    wait_lds();
    barrier();
    // p2: A[qm1]; stage Aq0(t+2)
    GG_T(6);
    read_a(buf, 1);
    stage_a(0, t + 2);
    wait_dma();
    barrier();
    GG_T(7);
    mma(1, 1);
    barrier();
    // p3: scale Aq0(t+1) (as in p1); rows for p0's stage; stage Bq0(t+2)
    GG_T(8);
    scale_load(nbuf, 0, t + 1);
    read_rows(1, t + 2);
    stage_b(0, t + 2);
    wait_dma();
    barrier();
    GG_T(9);
    mma(1, 0, true, nbuf, 0, t + 1);
    wait_lds();
    barrier();
    GG_T(10);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wr == 0) __builtin_amdgcn_s_barrier();  // match the staggered group's barrier count
  GG_AT(11);

  if (sizeof(OutT) == 2 && (epi & 15) != EPI_CROSS && ((N | int(ldc)) & 7) == 0)
    plain_staged_epilogue<false>(acc, smem, m0, n0, wr, wc, wid, lane, M, N, bias, nullptr, nullptr,
                                 reinterpret_cast<bf16*>(C), ldc, epi);
  else
    store_acc_t<false, false>(acc, m0 + 128 * wr, n0 + 64 * wc, fr, fq, M, N, bias, nullptr, nullptr, C, ldc, nullptr,
                              nullptr, 0, epi);
#ifdef DTFS_GG_STAMPS
  GG_AT(12);
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)
    for (int k = 0; k < 16; ++k) g_gg_stamps[blockIdx.x][threadIdx.x >> 6][k] = gg_s[k];
#endif
  if constexpr (EXTRA == 1) {
    if (fm_on) {
      float part = -fsq;
#pragma unroll
      for (int j = 0; j < 8; ++j) part += fs[j] * fs[j];
      part += __shfl_xor(part, 1, 64);
      part += __shfl_xor(part, 2, 64);
      part += __shfl_xor(part, 4, 64);
      if (sp_ch == 0) fm_part[Mp + m0 + scale_row(fm_q, fm_h)] = 0.5f * part;
    }
  } else if constexpr (EXTRA == 2) {
    if (fm_on) {  // x_l = alpha_l x0 + beta_l: alpha_{l+1} = alpha_l + alpha_l s_l + c_l
#pragma unroll
      for (int l = 0; l < XMAX; ++l) {
        fs[l] += __shfl_xor(fs[l], 1, 64);
        fs[l] += __shfl_xor(fs[l], 2, 64);
        fs[l] += __shfl_xor(fs[l], 4, 64);
      }
      const int L = cross_n - 1;
      float alpha = 1.f, dL = fs[0];
#pragma unroll
      for (int l = 0; l < XMAX; ++l) {
        if (l < L) alpha += alpha * fs[l] + cross_c[l];
        if (l == L) dL = fs[l];
      }
      if (sp_ch == 0) fm_part[Mp + m0 + scale_row(fm_q, fm_h)] = alpha * dL + cross_c[L];
    }
  }
}

// ---------------------------------------------------------------------------
// Deep-pipelined LDS-DMA variant: a STAGES-deep ring of K tiles with PREFETCH =
// STAGES - 1 tiles in flight across barriers (cdna_hip_programming.md §5
// "Pipelining across barriers"): every iteration issues the DMA for tile
// kt + PREFETCH, computes tile kt, then waits with a COUNTED vmcnt that leaves
// the just-issued tile in flight (never vmcnt(0) in the loop) and a raw
// s_barrier (not __syncthreads, whose fence would drain the DMA).
// Ring-slot hazards: slot (kt+P)%S was last read in iteration kt+P-S <= kt-1,
// which every wave finished before the barrier ending that iteration (WAR);
// tile kt+1 is read only after the vmcnt + barrier of iteration kt (RAW).
template <int BM, int BN, int WM_, int WN_, int STAGES, bool FP8, typename OutT>
__global__ void __launch_bounds__(WM_* WN_ * 64) gemm_pipe_kernel(
    const uint8_t* __restrict__ A, int64_t lda, const uint8_t* __restrict__ W, int64_t ldw,
    const float* __restrict__ bias, const float* __restrict__ sa, const float* __restrict__ sw, OutT* __restrict__ C,
    int64_t ldc, const bf16* __restrict__ X0, const bf16* __restrict__ XL, int64_t ldx, int M, int N, int K, int epi) {
  constexpr int NW = WM_ * WN_;
  constexpr int EB = FP8 ? 1 : 2;
  constexpr int WTM = BM / WM_, WTN = BN / WN_;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int IA = BM / 8 / NW, IB = BN / 8 / NW;  // LDS-DMA instructions per wave per tile
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "tile rows must split evenly over waves");
  constexpr int STAGE_BYTES = (BM + BN) * 128;
  constexpr int PF = STAGES - 1;
  constexpr int LOADS = IA + IB;

  __shared__ __attribute__((aligned(16))) uint8_t smem[STAGES * STAGE_BYTES];

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const bool m_fast = (epi & 16) != 0;
  const int tm = m_fast ? tile % tiles_m : tile / tiles_n;
  const int tn = m_fast ? tile / tiles_m : tile % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN_, wn = wid % WN_;

  const int lr = lane >> 3, ls = lane & 7;
  const uint8_t* a_src[IA];
  const uint8_t* b_src[IB];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int r = 8 * (wid + j * NW) + lr;
    a_src[j] = A + int64_t(min(m0 + r, M - 1)) * lda * EB + ((ls ^ ((r >> 1) & 7)) << 4);
  }
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int r = 8 * (wid + j * NW) + lr;
    b_src[j] = W + int64_t(min(n0 + r, N - 1)) * ldw * EB + ((ls ^ ((r >> 1) & 7)) << 4);
  }
  auto stage = [&](int slot, int kt) {
    uint8_t* base = smem + slot * STAGE_BYTES;
    const int64_t kb0 = int64_t(kt) * 128;
#pragma unroll
    for (int j = 0; j < IA; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(a_src[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + (wid + j * NW) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < IB; ++j)
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(b_src[j] + kb0),
                                       (__attribute__((address_space(3))) void*)(base + BM * 128 + (wid + j * NW) * 1024),
                                       16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K * EB) / 128;
  const int fr = lane & 15, fq = lane >> 4;
  // prologue: PF tiles in flight, tile 0 landed
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < nk) stage(p, p);
  if (nk > 1) {
    static_assert(PF <= 3, "extend the prologue wait ladder");
    // wait for tile 0 only: leave tiles 1..PF-1 (LOADS each) in flight
    if constexpr (PF == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
    else if constexpr (PF == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (nk < PF) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // short K: drain (rare)
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  for (int kt = 0; kt < nk; ++kt) {
    const int slot = kt % STAGES;
    const bool issue = kt + PF < nk;
    if (issue) stage((kt + PF) % STAGES, kt + PF);
    const uint8_t* as = smem + slot * STAGE_BYTES;
    const uint8_t* bs = as + BM * 128;
    if constexpr (!FP8) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(as + swz(wm * WTM + i * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8*>(bs + swz(wn * WTN + j * 16 + fr, kk * 4 + fq));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    } else {
      i32x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = mx_frag(as, wm * WTM + i * 16 + fr, fq);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = mx_frag(bs, wn * WTN + j * 16 + fr, fq);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mx_mfma(bfr[j], af[i], acc[i][j]);
    }
    // RAW for tile kt+1: this wave's loads for it are done once at most the
    // tiles issued after it are outstanding; every wave's, after the barrier.
    if (kt + 1 < nk) {
      const int ahead = min(PF - 1, nk - 1 - (kt + 1));  // tiles after kt+1 already issued
      if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
      else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this tile's ds_reads retired (WAR)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");  // keep the next tile's ds_reads below the barrier
    }
  }

  store_acc_t<FP8, false>(acc, m0 + wm * WTM, n0 + wn * WTN, fr, fq, M, N, bias, sa, sw, C, ldc, X0, XL, ldx, epi);
}

template <int BM, int BN, int WM_, int WN_, int STAGES, bool FP8, typename OutT>
static void launch_pipe(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                        const float* sw, OutT* C, int64_t ldc, const bf16* X0, const bf16* XL, int64_t ldx, int M,
                        int N, int K, int epi, hipStream_t st) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM_, WN_, STAGES, FP8, OutT>), dim3(grid), dim3(WM_ * WN_ * 64), 0, st,
                     static_cast<const uint8_t*>(A), lda, static_cast<const uint8_t*>(W), ldw, bias, sa, sw, C, ldc,
                     X0, XL, ldx, M, N, K, epi);
}

template <int BM, int BN, bool FP8, typename OutT>
static void launch_cfg(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                       const float* sw, OutT* C, int64_t ldc, const bf16* X0, const bf16* XL, int64_t ldx, int M, int N,
                       int K, int epi, hipStream_t st) {
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, FP8, OutT>), dim3(grid), dim3(256), 0, st,
                     static_cast<const uint8_t*>(A), lda, static_cast<const uint8_t*>(W), ldw, bias, sa, sw, C, ldc,
                     X0, XL, ldx, M, N, K, epi);
}

// Tile choice: the largest tile that still yields >= ~1 block per CU; small M
// (one request's worth of candidates) drops to 64x64 or 32x64 tiles.
template <bool FP8, typename OutT>
static void dispatch(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                     const float* sw, OutT* C, int64_t ldc, const bf16* X0, const bf16* XL, int64_t ldx, int M, int N,
                     int K, int epi, hipStream_t st, int variant, const MxIO& mx) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  const int EB = FP8 ? 1 : 2;
  // the LDS-DMA / 8-phase kernels need whole 128-byte K tiles and N % 4 == 0
  // (their epilogue stores 4 columns per lane; ragged N -> register-staged)
  const bool glds_ok = (K * EB) % 128 == 0 && N % 4 == 0;
  if constexpr (FP8) {
  if (mx.sab || mx.q) {
    // block-scaled activations in / out: the LDS-DMA kernels (32-column-aligned
    // wave tiles, a barrier per K tile so the scale-byte loads need no counting)
    const bool big = blocks(128, 128) >= 512;
#define DTFS_MX_LAUNCH(MXM)                                                                                         \
  (big ? launch_glds<128, 128, 2, 4, FP8, MXM>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st, \
                                               mx)                                                                  \
       : launch_glds<64, 64, 2, 2, FP8, MXM>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st, mx))
    if (mx.sab && mx.q) DTFS_MX_LAUNCH(3);
    else if (mx.sab) DTFS_MX_LAUNCH(1);
    else DTFS_MX_LAUNCH(2);
#undef DTFS_MX_LAUNCH
    return;
  }
  }
  const bool pre_from_dispatch = variant == 0;  // an explicit 17 keeps the plain kernel (A/B, tests)
  if (variant == 0 && glds_ok) {
    // The five tile variants kept (round-1/2 interleaved A/B sweeps, bench/
    // microbench.py --variants; 11 other tilings measured slower everywhere were
    // removed):
    //  *  8: M <= 1024 (one request's candidates): 64x64, 4-deep LDS ring
    //  * 17: >= 256 whole 256x256 tiles: the 8-phase kernel (16384x1024x2752:
    //        81.8 us vs 87.2 for 8-wave 128x128); a ragged last column panel
    //        (N = 2752) or fewer tiles than CUs loses to 14
    //  * 14: >= 512 tiles of 128x128: 8 waves per block (2 per SIMD), 2 blocks/CU
    //        (46.1 us vs 48.9 for 4 waves at 8192x1024x2752; DeepFM's GEMM2
    //        16384x512x1024: 22.6 us vs 24.1 for one 128x256 or 256x128 tile
    //        per CU and 30.3 for the 8-phase 256x256, round 4)
    //  * 10: >= 512 tiles of 128x64 (8192 x 512: 15.5 us vs 16.9 for 64x64)
    //  *  4: otherwise (narrow N): 64x64 LDS-DMA
    // K not a multiple of one 128-byte K tile: the register-staged gemm_kernel.
    if (M <= 1024) variant = 8;
    // ragged N (2752) with a PLAIN fp8 epilogue (the split DCN-v2 cross GEMM):
    // 8-phase 124.7 us vs 147.6 us for 14 at 16384 x 2752 x 2816 (81.6 vs 84.0
    // at 8192 rows, bench/cross_split.py); with the cross epilogue 14 stays ahead
    else if (blocks(256, 256) >= 256 && (N % 256 == 0 || (FP8 && (epi & 15) != EPI_CROSS))) variant = 17;
    else if (blocks(128, 128) >= 512) variant = 14;
    else if (blocks(128, 64) >= 512) variant = 10;  // 8192 x 512: 15.5 us vs 16.9 (64x64)
    else variant = 4;
  }
  if (variant == 4 && glds_ok) {
    launch_glds<64, 64, 2, 2, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    return;
  }
  if (variant == 8 && glds_ok) {
    launch_pipe<64, 64, 2, 2, 4, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    return;
  }
  if (variant == 10 && glds_ok) {
    launch_glds<128, 64, 2, 2, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    return;
  }
  // 256x256 8-phase (staggered wave groups, counted vmcnt)
  // 17: the 8-phase kernel; 18: the same with the next tile's A[qm0] read in
  // phase 3 (LDS reads per phase 4/4/8/8 instead of 12/4/8/0): 16384x1024x2752
  // bf16 76.2-76.9 us vs 80.9-81.9 (interleaved, MI355X), so the default
  // 8-phase pick (variant 0 -> 17) runs it
  if ((variant == 17 || variant == 18) && glds_ok) {
    const bool pre = variant == 18 || (variant == 17 && pre_from_dispatch);
    if (pre) launch_8ph<FP8, OutT, true>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    else launch_8ph<FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    return;
  }
  if (variant == 14 && glds_ok) {
    launch_glds<128, 128, 2, 4, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
    return;
  }
  if (blocks(128, 128) >= 256)
    launch_cfg<128, 128, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
  else if (blocks(64, 128) >= 256)
    launch_cfg<64, 128, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
  else if (blocks(64, 64) >= 192)
    launch_cfg<64, 64, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
  else
    launch_cfg<32, 64, FP8>(A, lda, W, ldw, bias, sa, sw, C, ldc, X0, XL, ldx, M, N, K, epi, st);
}

}  // namespace kern

using namespace kern;


hipError_t launch_gemm_head(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int act,
                            const float* hw, float hbias, const float* extra, int out_act, float* y, int M, int N,
                            int K, hipStream_t st, int extra_n, int64_t extra_ld) {
  if (M == 0) return hipSuccess;
  if ((K * 2) % 128 != 0 || N > 256 || N <= 0 || extra_n < 1 || (extra_n > 1 && extra_ld < M))
    return hipErrorInvalidValue;
  const uint8_t* a = static_cast<const uint8_t*>(A);
  const uint8_t* w = static_cast<const uint8_t*>(W);
  // 32-row tiles give >= 256 workgroups at the bench batch (8192 rows)
  const bool small = M >= 4096;
  if (N > 128) {
    if (small)
      hipLaunchKernelGGL((gemm_head_kernel<32, 4>), dim3((M + 31) / 32), dim3(256), 0, st, a, lda, w, ldw, bias, act,
                         hw, hbias, extra, extra_n, extra_ld, out_act, y, M, N, K);
    else
      hipLaunchKernelGGL((gemm_head_kernel<64, 4>), dim3((M + 63) / 64), dim3(256), 0, st, a, lda, w, ldw, bias, act,
                         hw, hbias, extra, extra_n, extra_ld, out_act, y, M, N, K);
  } else if (N > 64) {
    hipLaunchKernelGGL((gemm_head_kernel<64, 2>), dim3((M + 63) / 64), dim3(256), 0, st, a, lda, w, ldw, bias, act, hw,
                       hbias, extra, extra_n, extra_ld, out_act, y, M, N, K);
  } else {
    hipLaunchKernelGGL((gemm_head_kernel<64, 1>), dim3((M + 63) / 64), dim3(256), 0, st, a, lda, w, ldw, bias, act, hw,
                       hbias, extra, extra_n, extra_ld, out_act, y, M, N, K);
  }
  return hipGetLastError();
}

hipError_t launch_gemm_gather(const void* table, int64_t V, const int32_t* rows_t, const float* wts_t, int64_t Mp,
                              int F, const void* W, const float* bias, void* C, int64_t ldc, float* fm_part, int M,
                              int N, int epi, hipStream_t st, const float* cross_w, const float* cross_c,
                              int cross_n) {
  if (M == 0) return hipSuccess;
  if (F < 1 || N <= 0 || N % 256 != 0 || Mp % 256 != 0 || Mp < M || V < 1 || V > (int64_t(1) << 31) ||
      ldc < N || ldc % 4 != 0 || (fm_part && N < 1024) || int64_t(N) * F * 128 >= (int64_t(1) << 31) || !table ||
      !rows_t || !wts_t || !W || !C)
    return hipErrorInvalidValue;
  if (cross_w && (!fm_part || !cross_c || cross_n < 1 || cross_n > 4)) return hipErrorInvalidValue;
  const int grid = int(Mp / 256) * (N / 256);
#define DTFS_GG(X)                                                                                                 \
  hipLaunchKernelGGL((gemm_gather_kernel<bf16, X>), dim3(grid), dim3(512), 0, st, static_cast<const uint8_t*>(table), \
                     int(V - 1), rows_t, wts_t, Mp, static_cast<const uint8_t*>(W), bias, static_cast<bf16*>(C), ldc,  \
                     fm_part, cross_w, cross_c, cross_n, M, N, F, epi)
  if (cross_w) DTFS_GG(2);
  else if (fm_part) DTFS_GG(1);
  else DTFS_GG(0);
#undef DTFS_GG
  return hipGetLastError();
}

hipError_t launch_cross_gemm_fp8(const CrossGemmArgs& g, hipStream_t st) {
  if (g.M == 0 || g.N == 0) return hipSuccess;
  const int M = g.M, N = g.N, K = g.K;
  if (K % 128 != 0 || N % 8 != 0 || N < 8 || g.lda < K || g.ldw < K || !g.X0 || !g.XL || g.ldx < N ||
      g.ldx % 8 != 0 || !g.sa || (!g.Z && !g.dot) || (g.Z && (g.ldz < N || g.ldz % 8 != 0)) ||
      (g.dot && (!g.hw || g.ldd < M)))
    return hipErrorInvalidValue;
  XsArgs xs;
  xs.hw = g.hw;
  xs.dot = g.dot;
  xs.ldd = g.ldd;
  const int grid = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL((gemm_8ph_kernel<true, bf16, true, true>), dim3(grid), dim3(512), 0, st,
                     static_cast<const uint8_t*>(g.A), g.lda, static_cast<const uint8_t*>(g.W), g.ldw, g.bias, g.sa,
                     g.sw, static_cast<bf16*>(g.Z), g.ldz, static_cast<const bf16*>(g.X0),
                     static_cast<const bf16*>(g.XL), g.ldx, M, N, K, int(EPI_CROSS), xs);
  return hipGetLastError();
}

hipError_t launch_gemm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                       const float* sw, void* C, int64_t ldc, bool out_f32, const void* X0, const void* XL,
                       int64_t ldx, int M, int N, int K, int epi, bool fp8, hipStream_t st, int variant,
                       const MxIO* mxp) {
  if (M == 0 || N == 0) return hipSuccess;
  if ((fp8 ? K % 16 : K % 8) != 0) return hipErrorInvalidValue;  // 16-byte row chunks
  const MxIO mx = mxp ? *mxp : MxIO();
  if ((mx.sab || mx.q) && (!fp8 || K % 128 != 0 || N % 4 != 0)) return hipErrorInvalidValue;
  if (mx.sab && (K / 32 > kern::kMxMaxKBlocks || mx.ldsab % 4 != 0 || reinterpret_cast<uintptr_t>(mx.sab) % 4 != 0))
    return hipErrorInvalidValue;
  if (mx.q && ((epi & 15) != EPI_CROSS || !mx.sq || N % 32 != 0 || mx.nq < N || mx.nq % 32 != 0))
    return hipErrorInvalidValue;
  const bf16* x0 = static_cast<const bf16*>(X0);
  const bf16* xl = static_cast<const bf16*>(XL);
  if (fp8) {
    if (out_f32) dispatch<true>(A, lda, W, ldw, bias, sa, sw, static_cast<float*>(C), ldc, x0, xl, ldx, M, N, K, epi, st, variant, mx);
    else dispatch<true>(A, lda, W, ldw, bias, sa, sw, static_cast<bf16*>(C), ldc, x0, xl, ldx, M, N, K, epi, st, variant, mx);
  } else {
    if (out_f32) dispatch<false>(A, lda, W, ldw, bias, sa, sw, static_cast<float*>(C), ldc, x0, xl, ldx, M, N, K, epi, st, variant, mx);
    else dispatch<false>(A, lda, W, ldw, bias, sa, sw, static_cast<bf16*>(C), ldc, x0, xl, ldx, M, N, K, epi, st, variant, mx);
  }
  return hipGetLastError();
}

}  // namespace dtfs

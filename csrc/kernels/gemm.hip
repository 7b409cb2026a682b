// K3b/K4/K6: dense towers on CDNA4 matrix cores.
//
//   C[m, n] = epilogue( sum_k A[m, k] * W[n, k] )       A: [M][K], W: [N][K]
//
// bf16 operands use v_mfma_f32_16x16x32_bf16; fp8 (OCP e4m3) operands use
// v_mfma_f32_16x16x32_fp8_fp8 with a per-row activation scale and a
// per-output-channel weight scale folded into the epilogue.
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
#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

typedef long fp8x8;  // 8 x e4m3 packed, the fp8 MFMA operand type

enum Epi { EPI_NONE = 0, EPI_RELU = 1, EPI_SIGMOID = 2, EPI_CROSS = 3 };

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

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
  const int tm = tile % tiles_m, tn = tile / tiles_m;
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
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
      // fp8: 4 MFMA k-steps of 32 per 128-element tile; lane reads 8 bytes at
      // byte 32*kk + 8*fq = chunk 2*kk + (fq>>1), half (fq&1).
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        fp8x8 af[TM], bfr[TN];
        const int ch = kk * 2 + (fq >> 1), hoff = (fq & 1) * 8;
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const fp8x8*>(as + swz(wm * WM + i * 16 + fr, ch) + hoff);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const fp8x8*>(bs + swz(wn * WN + j * 16 + fr, ch) + hoff);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // Epilogue. C/D layout (16x16): col = lane & 15, row = 4 * (lane >> 4) + r.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + fr;
    if (n >= N) continue;
    const float bn = bias ? bias[n] : 0.f;
    const float swn = sw ? sw[n] : 1.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WM + i * 16 + fq * 4 + r;
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (FP8) v *= swn * (sa ? sa[m] : 1.f);
        v += bn;
        if (epi == EPI_RELU) v = fmaxf(v, 0.f);
        else if (epi == EPI_SIGMOID) v = sigmoidf(v);
        else if (epi == EPI_CROSS) v = bf2f(X0[m * ldx + n]) * v + bf2f(XL[m * ldx + n]);
        if constexpr (sizeof(OutT) == 2) C[m * ldc + n] = f2bf(v);
        else C[m * ldc + n] = v;
      }
    }
  }
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
                     int K, int epi, hipStream_t st) {
  auto blocks = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
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

hipError_t launch_gemm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                       const float* sw, void* C, int64_t ldc, bool out_f32, const void* X0, const void* XL,
                       int64_t ldx, int M, int N, int K, int epi, bool fp8, hipStream_t st) {
  if (M == 0 || N == 0) return hipSuccess;
  if ((fp8 ? K % 16 : K % 8) != 0) return hipErrorInvalidValue;  // 16-byte row chunks
  const bf16* x0 = static_cast<const bf16*>(X0);
  const bf16* xl = static_cast<const bf16*>(XL);
  if (fp8) {
    if (out_f32) dispatch<true>(A, lda, W, ldw, bias, sa, sw, static_cast<float*>(C), ldc, x0, xl, ldx, M, N, K, epi, st);
    else dispatch<true>(A, lda, W, ldw, bias, sa, sw, static_cast<bf16*>(C), ldc, x0, xl, ldx, M, N, K, epi, st);
  } else {
    if (out_f32) dispatch<false>(A, lda, W, ldw, bias, sa, sw, static_cast<float*>(C), ldc, x0, xl, ldx, M, N, K, epi, st);
    else dispatch<false>(A, lda, W, ldw, bias, sa, sw, static_cast<bf16*>(C), ldc, x0, xl, ldx, M, N, K, epi, st);
  }
  return hipGetLastError();
}

}  // namespace dtfs

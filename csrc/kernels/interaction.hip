// Feature-interaction kernels: K3 DCN cross v1 (all layers fused, optionally
// fused with the cross half of the output head), K5 DLRM dot interaction on
// MFMA, K6 output head (GEMV + bias + extra logit + sigmoid), fp8 row
// quantisation for the fp8 towers.
#include "common.h"
#include "launchers.h"
#include "peer_lookup.h"

namespace dtfs {
namespace kern {

// ---------------------------------------------------------------- K3
// x_{l+1} = x0 * (x_l . w_l) + b_l + x_l   for l < L, one wave per row, the
// whole row (d <= 64 * 8 * MAXC) resident in registers across all layers.
// Outputs: out_x = x_L (bf16, optional); out_dot[b] = x_L . head_w (optional).
template <int MAXC>
__global__ void __launch_bounds__(256) cross_v1_kernel(const bf16* __restrict__ x0, int64_t ldx, int B, int d, int L,
                                                       const float* __restrict__ w, const float* __restrict__ bvec,
                                                       bf16* __restrict__ out_x, int64_t ldo,
                                                       const float* __restrict__ head_w, float* __restrict__ out_dot) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (row >= B) return;
  const int nch = d / 8;
  float a0[MAXC][8], al[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(x0 + row * ldx + ch * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) a0[c][j] = al[c][j] = bf2f(v[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) a0[c][j] = al[c][j] = 0.f;
    }
  }
  for (int l = 0; l < L; ++l) {
    const float* wl = w + int64_t(l) * d;
    const float* bl = bvec + int64_t(l) * d;
    float p = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        const float4 w0 = *reinterpret_cast<const float4*>(wl + ch * 8);
        const float4 w1 = *reinterpret_cast<const float4*>(wl + ch * 8 + 4);
        p += al[c][0] * w0.x + al[c][1] * w0.y + al[c][2] * w0.z + al[c][3] * w0.w;
        p += al[c][4] * w1.x + al[c][5] * w1.y + al[c][6] * w1.z + al[c][7] * w1.w;
      }
    }
    const float s = wave_sum(p);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        const float4 b0 = *reinterpret_cast<const float4*>(bl + ch * 8);
        const float4 b1 = *reinterpret_cast<const float4*>(bl + ch * 8 + 4);
        const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) al[c][j] = a0[c][j] * s + bb[j] + al[c][j];
      }
    }
  }
  float hd = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch >= nch) continue;
    if (out_x) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(al[c][j]);
      *reinterpret_cast<bf16x8*>(out_x + row * ldo + ch * 8) = o;
    }
    if (head_w) {
#pragma unroll
      for (int j = 0; j < 8; ++j) hd += al[c][j] * head_w[ch * 8 + j];
    }
  }
  if (out_dot) {
    hd = wave_sum(hd);
    if (lane == 0) out_dot[row] = hd;
  }
}

// ---------------------------------------------------------------- K5
// DLRM pairwise dot interaction for T+1 <= 32 vectors of D = 64:
//   X = [dense; emb_0 .. emb_{T-1}]  (32 x 64 after zero padding)
//   Z = X X^T  via 4 x v_mfma_f32_32x32x16_bf16 (A and B fragments are the
//   same registers: lane (r, h) holds X[r][16s + 8h .. +8] for k-step s)
//   out[b] = [dense (D) | Z[i][j] for i > j, row-major (T+1)T/2 | zero pad]
__global__ void __launch_bounds__(256) dot_interact_kernel(const bf16* __restrict__ dense, int64_t ldd,
                                                           const bf16* __restrict__ emb, int T, int B,
                                                           bf16* __restrict__ out, int64_t ldo, int out_cols,
                                                           const int64_t* __restrict__ emb_off,
                                                           const int64_t* __restrict__ emb_stride, int64_t emb_rows) {
  constexpr int D = 64;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= B) return;
  const int r = lane & 31, h = lane >> 5;
  const int nv = T + 1;
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 x = bf16x8{};
    const int k = 16 * s + 8 * h;
    if (r == 0) x = *reinterpret_cast<const bf16x8*>(dense + b * ldd + k);
    else if (r < nv) {
      // table map: the embedding all-to-all's [owner][row][slot] layout in place
      const int64_t er = emb_off ? min(max(emb_off[r - 1] + int64_t(b) * emb_stride[r - 1], int64_t(0)), emb_rows - 1)
                                 : int64_t(b) * T + (r - 1);
      x = *reinterpret_cast<const bf16x8*>(emb + er * D + k);
    }
    // f32_32x32x16_bf16 operand = 8 bf16
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, x, acc, 0, 0, 0);
  }
  bf16* o = out + b * ldo;
  // dense passthrough (lanes 0..7 copy 8 each)
  if (lane < D / 8)
    *reinterpret_cast<bf16x8*>(o + lane * 8) = *reinterpret_cast<const bf16x8*>(dense + b * ldd + lane * 8);
  // C layout (32x32): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5)
  const int col = lane & 31;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int rowi = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (rowi < nv && col < rowi) o[D + rowi * (rowi - 1) / 2 + col] = f2bf(acc[reg]);
  }
  // zero the padding columns so the next GEMM's K tail reads zeros
  const int used = D + nv * (nv - 1) / 2;
  for (int c = used + lane; c < out_cols; c += 64) o[c] = f2bf(0.f);
}

// K1 fused into K5: the DLRM dot interaction straight from the embedding
// tables (one-hot, local tables). The gather kernel wrote emb [B, T, 64] to
// HBM and dot_interact_kernel read it back (63 MB each way per 16384-row
// step at T = 30); here the wave of row b looks its T rows up itself:
// lane (r, h), r = 1..T, reads table row off[r-1] + id(b, r-1) mod m[r-1],
// all four 16-byte chunks issued before the first MFMA (4 KB of independent
// random reads in flight per wave). The output row (dense | lower triangle |
// zero pad) is assembled in LDS and written as 16-byte vectors instead of
// 2-byte scattered stores.
// With peer.cbase set, the rows come through the peer lookup (peer_lookup.h):
// table-wise shards read where they live, hot remote rows from the replica
// cache - the same one-kernel step at any number of ranks.
template <typename IdT>
__global__ void __launch_bounds__(256) dot_interact_gather_kernel(
    const bf16* __restrict__ dense, int64_t ldd, const bf16* __restrict__ table, int64_t table_rows,
    const IdT* __restrict__ ids, int64_t ldi, const int64_t* __restrict__ modulo_f,
    const int64_t* __restrict__ offset_f, int T, int B, bf16* __restrict__ out, int64_t ldo, int out_cols,
    const uint8_t* __restrict__ arena, int id_col0, PeerLookupArgs peer) {
  constexpr int D = 64;
  constexpr int ROWB = 4 * 2048;  // LDS bytes per block: 4 waves x one output row (<= 1024 columns)
  __shared__ __attribute__((aligned(16))) uint8_t lds[ROWB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * (blockDim.x / 64) + w;
  if (b >= B) return;
  const int r = lane & 31, h = lane >> 5;
  const int nv = T + 1;
  const bf16* src = nullptr;
  int hit = -1;
  int64_t key = 0;
  if (r >= 1 && r < nv) {
    const int t = r - 1;
    const int64_t m = peer.cbase ? peer.trows[t] : modulo_f[t];
    int64_t id = 0;
    if (arena) {  // the request arena's row b (K0 fused: no unpack pass); padding rows read id 0
      const ArenaRow ar = arena_row(arena, kArenaPayloadOff, b);
      float w;
      if (ar.ids) arena_feature(ar, id_col0 + t, id, w);
    } else {
      id = int64_t(ids[int64_t(b) * ldi + t]);
    }
    int64_t v = id % m;
    if (v < 0) v += m;
    if (peer.cbase) {
      src = peer_row(peer, cache_view(peer), t, v, hit);
      key = (int64_t(t) << 40) | v;
    } else {
      src = table + min(offset_f[t] + v, table_rows - 1) * D;
    }
  }
  if (peer.cbase) {  // wave-uniform branches; converged: the ballots see every lane
    if (peer_counted(peer, b)) peer_count(peer, hit, h == 0);  // lanes h = 1 repeat h = 0's rows
    if (peer.sample_every > 0 && peer_sampled(peer, b)) ring_push(peer, key, h == 0 && hit >= 0);
  }
  bf16x8 x[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 16 * s + 8 * h;
    x[s] = bf16x8{};
    if (r == 0) x[s] = *reinterpret_cast<const bf16x8*>(dense + int64_t(b) * ldd + k);
    else if (src) x[s] = *reinterpret_cast<const bf16x8*>(src + k);
  }
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[s], x[s], acc, 0, 0, 0);
  // assemble the row in this wave's LDS slice: [dense | lower triangle | zeros]
  bf16* o = reinterpret_cast<bf16*>(lds + w * (ROWB / 4));
  const int n8 = out_cols / 8;
  for (int c = lane; c < n8; c += 64) *reinterpret_cast<bf16x8*>(o + c * 8) = bf16x8{};
  __builtin_amdgcn_wave_barrier();
  if (lane < D / 8) *reinterpret_cast<bf16x8*>(o + lane * 8) = *reinterpret_cast<const bf16x8*>(dense + int64_t(b) * ldd + lane * 8);
  const int col = lane & 31;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) {
    const int rowi = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
    if (rowi < nv && col < rowi) o[D + rowi * (rowi - 1) / 2 + col] = f2bf(acc[reg]);
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bf16* dst = out + int64_t(b) * ldo;
  for (int c = lane; c < n8; c += 64) *reinterpret_cast<bf16x8*>(dst + c * 8) = *reinterpret_cast<const bf16x8*>(o + c * 8);
}

// ---------------------------------------------------------------- K4 (small)
// DLRM bottom MLP in one kernel: the dense features (fp32 columns [0, nd) of
// feat_wts) -> bf16, zero padded to K0 = 64 -> relu(. W1^T + b1) [N1] ->
// relu(. W2^T + b2) [N2] -> relu(. W3^T + b3) [N3] (bf16 out). Per block 32
// rows, every intermediate in LDS; the weights (~176 K bf16, L2-resident)
// are read as MFMA B fragments straight from global memory. As separate
// launches these are three small GEMMs + a pad kernel, each mostly launch /
// prologue / epilogue (~31 us per 16384-row step for 5.8 GFLOP).
// Layer layout: wave w owns output columns [w N / 4, (w + 1) N / 4); D = W_frag x
// A_frag^T, so lane (fr, fq) holds rows 16 i + fr, columns 4 fq .. 4 fq + 3 of
// each 16 x 16 tile. LDS row pitches are the row bytes + 16: the 16 rows of a
// ds_read_b128 lane group land on 16 distinct 16-byte bank slots.
template <int K, int NW, int PIN, int POUT>
__device__ __forceinline__ void mlp_layer_lds(const uint8_t* __restrict__ ain, const bf16* __restrict__ W,
                                              const float* __restrict__ b, uint8_t* __restrict__ hout,
                                              bf16* __restrict__ gout, int64_t ldo, int m0, int M, int wid, int fr,
                                              int fq) {
  constexpr int TN = NW / 16;
  f32x4 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int n0 = wid * NW;
#pragma unroll 4
  for (int s = 0; s < K / 32; ++s) {
    bf16x8 a[2], w[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      w[j] = *reinterpret_cast<const bf16x8*>(W + int64_t(n0 + 16 * j + fr) * K + 32 * s + 8 * fq);
#pragma unroll
    for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(ain + (16 * i + fr) * PIN + (32 * s + 8 * fq) * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], a[i], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + 16 * j + 4 * fq;
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(b + n);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = f2bf(fmaxf(acc[i][j][r] + b4[r], 0.f));
      const int row = 16 * i + fr;
      if (gout) {
        if (m0 + row < M) *reinterpret_cast<bf16x4*>(gout + int64_t(m0 + row) * ldo + n) = o;
      } else {
        *reinterpret_cast<bf16x4*>(hout + row * POUT + n * 2) = o;
      }
    }
  }
}

template <int N1, int N2, int N3>
__global__ void __launch_bounds__(256) bottom_mlp3_kernel(const float* __restrict__ wts, int64_t ldw, int nd, int M,
                                                          const bf16* __restrict__ W1, const float* __restrict__ b1,
                                                          const bf16* __restrict__ W2, const float* __restrict__ b2,
                                                          const bf16* __restrict__ W3, const float* __restrict__ b3,
                                                          bf16* __restrict__ out, int64_t ldo,
                                                          const uint8_t* __restrict__ arena) {
  constexpr int BM = 32, K0 = 64;
  constexpr int PX = K0 * 2 + 16, P1 = N1 * 2 + 16, P2 = N2 * 2 + 16;
  __shared__ __attribute__((aligned(16))) uint8_t lds[BM * (PX + P1 + P2)];
  uint8_t* X = lds;
  uint8_t* H1 = X + BM * PX;
  uint8_t* H2 = H1 + BM * P1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const int m0 = blockIdx.x * BM;
  {  // X: thread t -> row t / 8, columns 8 (t % 8) .. +8 (fp32 -> bf16, zero pad)
    const int row = threadIdx.x >> 3, c0 = (threadIdx.x & 7) * 8;
    const int64_t m = min(m0 + row, M - 1);
    bf16x8 v;
    if (arena) {  // dense features = the first nd weights of the arena row (padding rows: 0)
      const ArenaRow ar = arena_row(arena, kArenaPayloadOff, m);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        int64_t id;
        float w = 0.f;
        if (ar.ids && c0 + e < nd) arena_feature(ar, c0 + e, id, w);
        v[e] = f2bf(w);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(c0 + e < nd ? wts[m * ldw + c0 + e] : 0.f);
    }
    *reinterpret_cast<bf16x8*>(X + row * PX + c0 * 2) = v;
  }
  __syncthreads();
  mlp_layer_lds<K0, N1 / 4, PX, P1>(X, W1, b1, H1, nullptr, 0, m0, M, wid, fr, fq);
  __syncthreads();
  mlp_layer_lds<N1, N2 / 4, P1, P2>(H1, W2, b2, H2, nullptr, 0, m0, M, wid, fr, fq);
  __syncthreads();
  mlp_layer_lds<N2, N3 / 4, P2, 0>(H2, W3, b3, nullptr, out, ldo, m0, M, wid, fr, fq);
}

// ---------------------------------------------------------------- K6
// y[m] = act(x[m,:] . w + bias + extra[m]); one wave per row; act: 0 none, 2 sigmoid.
__global__ void __launch_bounds__(256) head_kernel(const bf16* __restrict__ x, int64_t ldx, const float* __restrict__ w,
                                                   float bias, const float* __restrict__ extra, int extra_n,
                                                   int64_t extra_ld, int M, int K, int act, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  float p = 0.f;
  for (int ch = lane; ch < K / 8; ch += 64) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + m * ldx + ch * 8);
    const float4 w0 = *reinterpret_cast<const float4*>(w + ch * 8);
    const float4 w1 = *reinterpret_cast<const float4*>(w + ch * 8 + 4);
    p += bf2f(v[0]) * w0.x + bf2f(v[1]) * w0.y + bf2f(v[2]) * w0.z + bf2f(v[3]) * w0.w;
    p += bf2f(v[4]) * w1.x + bf2f(v[5]) * w1.y + bf2f(v[6]) * w1.z + bf2f(v[7]) * w1.w;
  }
  p = wave_sum(p);
  if (lane == 0) {
    float v = p + bias;
    for (int e = 0; extra && e < extra_n; ++e) v += extra[e * extra_ld + m];
    out[m] = act == 2 ? sigmoidf(v) : v;
  }
}

// ---------------------------------------------------------------- DLRM dense input
// y[b, :] = bf16(x[b, 0 .. n)) zero padded to K columns, one 16-byte store per
// thread (replaces torch.zeros + a strided cast-copy: two kernels, ~17 us of
// the served 16384-row DLRM step under the H2D copy).
__global__ void __launch_bounds__(256) dense_pad_kernel(const float* __restrict__ x, int64_t ldx, int M, int n,
                                                        bf16* __restrict__ y, int K) {
  const int cpr = K / 8;
  const int64_t c = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (c >= int64_t(M) * cpr) return;
  const int64_t b = c / cpr;
  const int j0 = int(c - b * cpr) * 8;
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(j0 + j < n ? x[b * ldx + j0 + j] : 0.f);
  *reinterpret_cast<bf16x8*>(y + b * K + j0) = o;
}

// ---------------------------------------------------------------- fp8 quant
// Per-row dynamic e4m3 quantisation: scale = amax / 448, q = x / scale.
template <int MAXC>
__global__ void __launch_bounds__(256) quant_rows_kernel(const bf16* __restrict__ x, int64_t ldx, int M, int K,
                                                         uint8_t* __restrict__ q, int64_t ldq, float* __restrict__ scale,
                                                         int Kq) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const int nch = K / 8;
  // zero the K padding (columns [K, Kq)) the 128-deep fp8 MFMA tiles read
  for (int ch = nch + lane; ch < Kq / 8; ch += 64) *reinterpret_cast<int2*>(q + m * ldq + ch * 8) = make_int2(0, 0);
  float v[MAXC][8];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const bf16x8 t = *reinterpret_cast<const bf16x8*>(x + m * ldx + ch * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = bf2f(t[j]);
        amax = fmaxf(amax, fabsf(v[c][j]));
      }
    }
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[m] = s;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      int lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][0] * inv, v[c][1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][2] * inv, v[c][3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4] * inv, v[c][5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][6] * inv, v[c][7] * inv, hi, true);
      *reinterpret_cast<int2*>(q + m * ldq + ch * 8) = make_int2(lo, hi);
    }
  }
}

// The same quantisation, each lane owning 16 consecutive columns (two 16-byte
// loads, ONE 16-byte store of 16 e4m3 values instead of two 8-byte ones);
// K, Kq multiples of 16, 16-byte aligned rows. Bit-equal to quant_rows_kernel.
template <int MAXP>
__global__ void __launch_bounds__(256) quant_rows16_kernel(const bf16* __restrict__ x, int64_t ldx, int M, int K,
                                                           uint8_t* __restrict__ q, int64_t ldq,
                                                           float* __restrict__ scale, int Kq) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const int np = K / 16;
  for (int p = np + lane; p < Kq / 16; p += 64) *reinterpret_cast<int4*>(q + m * ldq + p * 16) = make_int4(0, 0, 0, 0);
  float v[MAXP][16];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < MAXP; ++c) {
    const int p = lane + c * 64;
    if (p < np) {
      const bf16x8 t0 = *reinterpret_cast<const bf16x8*>(x + m * ldx + p * 16);
      const bf16x8 t1 = *reinterpret_cast<const bf16x8*>(x + m * ldx + p * 16 + 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = bf2f(t0[j]);
        v[c][j + 8] = bf2f(t1[j]);
        amax = fmaxf(amax, fmaxf(fabsf(v[c][j]), fabsf(v[c][j + 8])));
      }
    }
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[m] = s;
#pragma unroll
  for (int c = 0; c < MAXP; ++c) {
    const int p = lane + c * 64;
    if (p < np) {
      int o[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        o[d] = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4 * d] * inv, v[c][4 * d + 1] * inv, 0, false);
        o[d] = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4 * d + 2] * inv, v[c][4 * d + 3] * inv, o[d], true);
      }
      *reinterpret_cast<int4*>(q + m * ldq + p * 16) = make_int4(o[0], o[1], o[2], o[3]);
    }
  }
}

// DCN-v2 cross combine, the second half of a split cross layer: the GEMM
// writes y = xl W^T + b (plain bf16 epilogue, so the big 8-phase tile can run
// it), then one wave per row computes z = x0 * y + xl (fp32, rounded to bf16)
// and, in the same pass over the row,
//   * writes z (the next layer's xl) and/or
//   * quantises z to e4m3 with a per-row scale (the next layer's fp8 operand,
//     zero-padded to Kq columns; same rounding as quant_rows_kernel) and/or
//   * reduces dot[m] = z . head_w (the last layer: z never reaches memory).
// Measured at 16384 x 2752 x 2816 fp8 (bench/cross_split.py, MI355X): fused
// cross epilogue 215.6 us + quant_rows 22.8 us vs plain 8-phase GEMM 124.7 us
// + a 360 MB elementwise pass ~63 us.
template <int MAXC>
__global__ void __launch_bounds__(256) cross_combine_kernel(const bf16* __restrict__ y, const bf16* __restrict__ x0,
                                                            const bf16* __restrict__ xl, int64_t ld, int M, int N,
                                                            bf16* __restrict__ z, int64_t ldz, uint8_t* __restrict__ q,
                                                            int64_t ldq, float* __restrict__ scale, int Kq,
                                                            const float* __restrict__ head_w, float* __restrict__ dot) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (m >= M) return;
  const int nch = N / 8;
  // the first cross layer's residual is x0 itself: read it once (a fifth of
  // that pass's HBM bytes)
  const bool xl_is_x0 = xl == x0;
  float v[MAXC][8];
  float amax = 0.f, acc = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      const int64_t o = int64_t(m) * ld + ch * 8;
      const bf16x8 ty = *reinterpret_cast<const bf16x8*>(y + o);
      const bf16x8 t0 = *reinterpret_cast<const bf16x8*>(x0 + o);
      const bf16x8 tl = xl_is_x0 ? t0 : *reinterpret_cast<const bf16x8*>(xl + o);
      bf16x8 tz;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        tz[j] = f2bf(bf2f(t0[j]) * bf2f(ty[j]) + bf2f(tl[j]));
        v[c][j] = bf2f(tz[j]);  // quantise / reduce exactly what the next layer would read back
        amax = fmaxf(amax, fabsf(v[c][j]));
      }
      if (z) *reinterpret_cast<bf16x8*>(z + int64_t(m) * ldz + ch * 8) = tz;
      if (head_w) {
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(head_w + ch * 8);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(head_w + ch * 8 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc += v[c][j] * w0[j] + v[c][j + 4] * w1[j];
      }
    }
  }
  if (head_w) {
    acc = wave_sum(acc);
    if (lane == 0) dot[m] = acc;
  }
  if (!q) return;
  for (int ch = nch + lane; ch < Kq / 8; ch += 64) *reinterpret_cast<int2*>(q + m * ldq + ch * 8) = make_int2(0, 0);
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[m] = s;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      int lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][0] * inv, v[c][1] * inv, lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][2] * inv, v[c][3] * inv, lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][4] * inv, v[c][5] * inv, hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[c][6] * inv, v[c][7] * inv, hi, true);
      *reinterpret_cast<int2*>(q + m * ldq + ch * 8) = make_int2(lo, hi);
    }
  }
}

}  // namespace kern

using namespace kern;

hipError_t launch_cross_combine(const void* y, const void* x0, const void* xl, int64_t ld, int M, int N, void* z,
                                int64_t ldz, void* q, int64_t ldq, float* scale, int Kq, const float* head_w,
                                float* dot, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (N % 8 || ld < N || (z && ldz < N) || (q && (Kq % 8 || Kq < N || ldq < Kq || !scale)) || (head_w && !dot))
    return hipErrorInvalidValue;
  const int chunks = (N / 8 + 63) / 64;
  dim3 grid((M + 3) / 4), block(256);
  const bf16* yi = static_cast<const bf16*>(y);
  const bf16* x0i = static_cast<const bf16*>(x0);
  const bf16* xli = static_cast<const bf16*>(xl);
  bf16* zo = static_cast<bf16*>(z);
  uint8_t* qo = static_cast<uint8_t*>(q);
#define CC_CASE(C)                                                                                              \
  case C:                                                                                                      \
    hipLaunchKernelGGL(cross_combine_kernel<C>, grid, block, 0, st, yi, x0i, xli, ld, M, N, zo, ldz, qo, ldq, scale, \
                       Kq, head_w, dot);                                                                       \
    break;
  switch (chunks) {
    CC_CASE(1) CC_CASE(2) CC_CASE(3) CC_CASE(4) CC_CASE(5) CC_CASE(6) CC_CASE(7) CC_CASE(8)
    default: return hipErrorInvalidValue;
  }
#undef CC_CASE
  return hipGetLastError();
}

hipError_t launch_cross_v1(const void* x0, int64_t ldx, int B, int d, int L, const float* w, const float* b,
                           void* out_x, int64_t ldo, const float* head_w, float* out_dot, hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (d % 8) return hipErrorInvalidValue;
  const int chunks = (d / 8 + 63) / 64;
  dim3 grid((B + 3) / 4), block(256);
  const bf16* xi = static_cast<const bf16*>(x0);
  bf16* xo = static_cast<bf16*>(out_x);
#define CROSS_CASE(C)                                                                                          \
  case C:                                                                                                     \
    hipLaunchKernelGGL(cross_v1_kernel<C>, grid, block, 0, st, xi, ldx, B, d, L, w, b, xo, ldo, head_w, out_dot); \
    break;
  switch (chunks) {
    CROSS_CASE(1) CROSS_CASE(2) CROSS_CASE(3) CROSS_CASE(4) CROSS_CASE(5) CROSS_CASE(6) CROSS_CASE(7) CROSS_CASE(8)
    default: return hipErrorInvalidValue;
  }
#undef CROSS_CASE
  return hipGetLastError();
}

hipError_t launch_dot_interaction(const void* dense, int64_t ldd, const void* emb, int T, int B, void* out,
                                  int64_t ldo, int out_cols, hipStream_t st, const int64_t* emb_off,
                                  const int64_t* emb_stride, int64_t emb_rows) {
  if (B == 0) return hipSuccess;
  if (emb_off && emb_rows < 1) return hipErrorInvalidValue;
  if (T + 1 > 32) return hipErrorInvalidValue;
  if ((emb_off == nullptr) != (emb_stride == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dot_interact_kernel, dim3((B + 3) / 4), dim3(256), 0, st, static_cast<const bf16*>(dense), ldd,
                     static_cast<const bf16*>(emb), T, B, static_cast<bf16*>(out), ldo, out_cols, emb_off, emb_stride, emb_rows);
  return hipGetLastError();
}

hipError_t launch_dot_interaction_gather(const void* dense, int64_t ldd, const void* table, int64_t table_rows,
                                         const void* ids, bool ids64, int64_t ldi, const int64_t* modulo_f,
                                         const int64_t* offset_f, int T, int B, void* out, int64_t ldo, int out_cols,
                                         hipStream_t st, const void* arena, int id_col0,
                                         const PeerLookupArgs* peer) {
  if (B == 0) return hipSuccess;
  const bool pl = peer && peer->cbase;
  if (T < 1 || T + 1 > 32 || out_cols % 8 || out_cols > 1024 || out_cols < 64 + (T + 1) * T / 2 || ldo % 8 ||
      ldo < out_cols || ldd % 8 || (!arena && (!ids || ldi < T)) || (arena && id_col0 < 0) ||
      (!pl && (table_rows < 1 || !modulo_f || !offset_f)) || (pl && (!peer->trows || !peer->tremote || !peer->towner || !peer->toff || peer->max_chunks < 1 ||
              peer->chunk_shift < 1 || peer->chunk_shift > 40)))
    return hipErrorInvalidValue;
  const PeerLookupArgs pa = pl ? *peer : PeerLookupArgs{};
  const uint8_t* ar = static_cast<const uint8_t*>(arena);
  dim3 grid((B + 3) / 4), block(256);
  if (ids64)
    hipLaunchKernelGGL(dot_interact_gather_kernel<int64_t>, grid, block, 0, st, static_cast<const bf16*>(dense), ldd,
                       static_cast<const bf16*>(table), table_rows, static_cast<const int64_t*>(ids), ldi, modulo_f,
                       offset_f, T, B, static_cast<bf16*>(out), ldo, out_cols, ar, id_col0, pa);
  else
    hipLaunchKernelGGL(dot_interact_gather_kernel<int32_t>, grid, block, 0, st, static_cast<const bf16*>(dense), ldd,
                       static_cast<const bf16*>(table), table_rows, static_cast<const int32_t*>(ids), ldi, modulo_f,
                       offset_f, T, B, static_cast<bf16*>(out), ldo, out_cols, ar, id_col0, pa);
  return hipGetLastError();
}

hipError_t launch_bottom_mlp3(const float* wts, int64_t ldw, int nd, int M, const void* W1, const float* b1, int N1,
                              const void* W2, const float* b2, int N2, const void* W3, const float* b3, int N3,
                              void* out, int64_t ldo, hipStream_t st, const void* arena) {
  if (M == 0) return hipSuccess;
  if (nd < 1 || nd > 64 || (!arena && (!wts || ldw < nd)) || ldo < N3 || ldo % 4 || !W1 || !W2 || !W3 || !b1 ||
      !b2 || !b3)
    return hipErrorInvalidValue;
  if (N1 == 512 && N2 == 256 && N3 == 64) {  // DLRM bottom_mlp [512, 256, 64]
    hipLaunchKernelGGL((bottom_mlp3_kernel<512, 256, 64>), dim3((M + 31) / 32), dim3(256), 0, st, wts, ldw, nd, M,
                       static_cast<const bf16*>(W1), b1, static_cast<const bf16*>(W2), b2,
                       static_cast<const bf16*>(W3), b3, static_cast<bf16*>(out), ldo,
                       static_cast<const uint8_t*>(arena));
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

hipError_t launch_head(const void* x, int64_t ldx, const float* w, float bias, const float* extra, int M, int K,
                       int act, float* out, hipStream_t st, int extra_n, int64_t extra_ld) {
  if (M == 0) return hipSuccess;
  if (K % 8 || extra_n < 1 || (extra_n > 1 && extra_ld < M)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_kernel, dim3((M + 3) / 4), dim3(256), 0, st, static_cast<const bf16*>(x), ldx, w, bias,
                     extra, extra_n, extra_ld, M, K, act, out);
  return hipGetLastError();
}

hipError_t launch_dense_pad(const float* x, int64_t ldx, int M, int n, void* y, int K, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (K % 8 || n > K || n < 0 || ldx < n) return hipErrorInvalidValue;
  const int64_t chunks = int64_t(M) * (K / 8);
  hipLaunchKernelGGL(dense_pad_kernel, dim3(unsigned((chunks + 255) / 256)), dim3(256), 0, st, x, ldx, M, n,
                     static_cast<bf16*>(y), K);
  return hipGetLastError();
}

hipError_t launch_quant_rows_fp8(const void* x, int64_t ldx, int M, int K, void* q, int64_t ldq, float* scale,
                                 hipStream_t st, int Kq) {
  if (M == 0) return hipSuccess;
  if (Kq <= 0) Kq = K;
  if (K % 8 || Kq % 8 || Kq < K || ldq < Kq) return hipErrorInvalidValue;
  dim3 grid((M + 3) / 4), block(256);
  const bf16* xi = static_cast<const bf16*>(x);
  uint8_t* qo = static_cast<uint8_t*>(q);
  // 16 columns per lane when the rows allow 16-byte accesses: bit-equal, 21.5 vs
  // 22.9 us at 16384 x 2752 (tools/native/quant_ab.hip)
  const int pairs = (K / 16 + 63) / 64;
  if (K % 16 == 0 && Kq % 16 == 0 && ldx % 8 == 0 && ldq % 16 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(q) % 16 == 0 && pairs >= 1 && pairs <= 4) {
#define Q16_CASE(C)                                                                                       \
  case C: hipLaunchKernelGGL(quant_rows16_kernel<C>, grid, block, 0, st, xi, ldx, M, K, qo, ldq, scale, Kq); break;
    switch (pairs) { Q16_CASE(1) Q16_CASE(2) Q16_CASE(3) Q16_CASE(4) }
#undef Q16_CASE
    return hipGetLastError();
  }
  const int chunks = (K / 8 + 63) / 64;
#define Q_CASE(C)                                                                                   \
  case C: hipLaunchKernelGGL(quant_rows_kernel<C>, grid, block, 0, st, xi, ldx, M, K, qo, ldq, scale, Kq); break;
  switch (chunks) {
    Q_CASE(1) Q_CASE(2) Q_CASE(3) Q_CASE(4) Q_CASE(5) Q_CASE(6) Q_CASE(7) Q_CASE(8)
    default: return hipErrorInvalidValue;
  }
#undef Q_CASE
  return hipGetLastError();
}

}  // namespace dtfs

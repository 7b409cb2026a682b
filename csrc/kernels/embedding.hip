// Sparse side of the CTR forward: K0 input packing, K1 weighted embedding
// gather (+ fused FM / first-order terms), K1b embedding-bag pooling.
//
// The reference only shows the tensors the client sends to this compute
// (feat_ids int64 [B,43], feat_wts fp32 [B,43]; reference DCNClient.java:97-108);
// the math below is the implied TF-Serving DCN/DeepFM graph.
//
// K1 layout: one wave per candidate row. With D = 64 a table row is 128 B = 8
// lanes x 16 B, so one wave-wide load instruction fetches 8 fields' rows; the
// ids/weights of the whole row are loaded once (lane f holds field f) and
// broadcast with __shfl, so each wave has exactly two dependent memory round
// trips (ids, then every table row at once) regardless of the field count.
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace dtfs {
namespace kern {

// ---------------------------------------------------------------- K0
template <typename IdT>
__global__ void __launch_bounds__(256) pack_ids_kernel(const IdT* __restrict__ ids, int32_t* __restrict__ out,
                                                       int64_t n, int F, const int64_t* __restrict__ modulo_f,
                                                       const int64_t* __restrict__ offset_f, int64_t modulo) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int f = int(i % F);
    const int64_t m = modulo_f ? modulo_f[f] : modulo;
    const int64_t off = offset_f ? offset_f[f] : 0;
    out[i] = int32_t(off + hash_row(int64_t(ids[i]), m));
  }
}

// ---------------------------------------------------------------- K1
// out_x[b, f*D + d] = table[row(b,f), d] * wts[b,f]              (bf16)
// out_fm[b] = bias + sum_f lin[row]*w  (first order, if lin)
//           + 0.5 * sum_d ((sum_f e)^2 - sum_f e^2)  (second order, if fm2)
// ids / wts may be strided row views (ids_ld / wts_ld elements per row), so a
// packed request row [ids int64 x F | wts fp32 x F | pad] is read in place.
// FM logit of one row from per-lane partial sums (lane = field group `sub`
// x dims dl..dl+7): returns sum over the wave of
//   0.5 * (sum_d S_d^2 - sum_{f,d} e^2) + first      (S_d = sum_f e[f, d])
// S_d needs a cross-lane sum over the field groups (lane bits log2(LPR)..5)
// per dim. Instead of an all-reduce of all 8 dims per step (24 shuffles at
// D = 64), each xor step exchanges only half of the values still held, so
// a lane ends up owning the full sums of 8 >> steps dims (7 shuffles at
// D = 64); sum e^2 needs no per-dim sums at all and rides on the final
// wave_sum together with the first-order term.
template <int LPR>
__device__ __forceinline__ float fm_row_logit(const float (&s)[8], const float (&q)[8], float first, bool fm2,
                                              int lane) {
  float part = first;
  if (fm2) {
    float cur[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) cur[j] = s[j];
    int width = 8;
    bool dup = false;  // lanes that hold a copy of another lane's sums (counted once)
#pragma unroll
    for (int off = kWave / 2; off >= LPR; off >>= 1) {
      const bool hb = (lane & off) != 0;
      if (width > 1) {
        const int half = width / 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < half) {
            const float keep = hb ? cur[half + k] : cur[k];
            const float give = hb ? cur[k] : cur[half + k];
            cur[k] = keep + __shfl_xor(give, off, kWave);
          }
        }
        width = half;
      } else {
        cur[0] += __shfl_xor(cur[0], off, kWave);
        dup = dup || hb;
      }
    }
    float sq = 0.f, qs = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < width) sq += cur[k] * cur[k];
#pragma unroll
    for (int j = 0; j < 8; ++j) qs += q[j];
    part += 0.5f * ((dup ? 0.f : sq) - qs);
  }
  return wave_sum(part);
}

// feature weight: fp32, or bf16 rows (narrow packed rows of the fan-out); 1 without weights
__device__ __forceinline__ float load_weight(const EmbedArgs& a, int64_t i) {
  if (!a.wts) return 1.f;
  if (a.wts16) return __uint_as_float(uint32_t(static_cast<const uint16_t*>(a.wts)[i]) << 16);
  return static_cast<const float*>(a.wts)[i];
}

template <int D, typename IdT, bool ARENA>
__global__ void __launch_bounds__(256) embed_kernel(EmbedArgs a) {
  constexpr int LPR = D / 8;          // lanes per table row (16 B each)
  constexpr int FPI = kWave / LPR;    // fields per wave-wide load
  const bf16* __restrict__ table = static_cast<const bf16*>(a.table);
  const IdT* __restrict__ ids = static_cast<const IdT*>(a.ids);
  const int F = a.F;
  const int lane = threadIdx.x & 63;
  const int b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (b >= a.B) return;
  ArenaRow arow{nullptr, nullptr};
  if constexpr (ARENA) arow = arena_row(static_cast<const uint8_t*>(a.arena), kArenaPayloadOff, b);
  const int sub = lane / LPR;         // which field of the instruction group
  const int dl = (lane % LPR) * 8;    // first dim this lane owns

  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  float first = 0.f;

  for (int fbase = 0; fbase < F; fbase += kWave) {
    // lane f loads field (fbase+f)'s id / weight
    const int fl = fbase + lane;
    int64_t row = 0;
    float w = 0.f;
    if (fl < F) {
      int64_t id;
      float w_in;
      if constexpr (ARENA) {  // padding rows (no request): id 0, weight 0 -> zero contribution
        id = 0;
        w_in = 0.f;
        if (arow.ids) arena_feature(arow, fl, id, w_in);
      } else {
        id = int64_t(ids[int64_t(b) * a.ids_ld + fl]);
        w_in = load_weight(a, int64_t(b) * a.wts_ld + fl);
      }
      const int64_t m = a.modulo_f ? a.modulo_f[fl] : a.modulo;
      int64_t g = hash_row(id, m);
      bool own = true;
      if (a.shard_lo_f) {
        g -= a.shard_lo_f[fl];
        own = g >= 0 && g < a.shard_n_f[fl];
        g = own ? g : 0;
      }
      row = (a.offset_f ? a.offset_f[fl] : 0) + g;
      row = row < 0 ? 0 : (row >= a.V ? a.V - 1 : row);  // memory safety whatever the tables say
      w = own ? w_in : 0.f;
      if (a.lin) first += a.lin[row] * w;
    }
    const int nf = min(kWave, F - fbase);
    const int groups = (nf + FPI - 1) / FPI;
    // Issue every table load of this chunk before consuming any.
    constexpr int MAXG = kWave / FPI;  // 8 for D=64
    bf16x8 v[MAXG];
    float wf[MAXG];
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      const int f = g * FPI + sub;
      const int64_t r = __shfl(row, min(f, kWave - 1), 64);
      wf[g] = __shfl(w, min(f, kWave - 1), 64);
      if (g < groups && f < nf) {
        v[g] = *reinterpret_cast<const bf16x8*>(table + r * D + dl);
      } else {
        v[g] = bf16x8{};
        wf[g] = 0.f;
      }
    }
    bf16* __restrict__ out_x = static_cast<bf16*>(a.out_x);
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      const int f = g * FPI + sub;
      if (g < groups && f < nf) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = bf2f(v[g][j]) * wf[g];
          s[j] += e;
          q[j] += e * e;
          o[j] = f2bf(e);
        }
        if (out_x) *reinterpret_cast<bf16x8*>(out_x + int64_t(b) * a.x_ld + int64_t(fbase + f) * D + dl) = o;
      }
    }
  }

  if (!a.out_fm) return;
  const float logit = fm_row_logit<LPR>(s, q, first, a.fm2 != 0, lane);
  if (lane == 0) a.out_fm[b] = a.bias + logit;
}

// ---------------------------------------------------------------- K1 (pipelined)
// Same math as embed_kernel for F <= 64, restructured for the serving shape
// (thousands of rows, Zipf ids, table mostly cache-resident). There the
// one-row-per-wave kernel is bound by each wave's chain of dependent memory
// round trips (arena row table -> ids/weights -> table rows -> stores), not
// by bandwidth: measured 40.5 us for 16384 x 43 rows vs a 14 us write floor.
// Here a wave walks rows b, b + nwaves, ... and issues row b+nwaves' id /
// weight loads right behind row b's table loads, so from the second row on
// the id fetch hides under the gather. The id -> row hash uses a multiply-high
// reciprocal (host-computed) instead of the 64-bit software modulo.

// (hash_row_magic: common.h)

// K3 in the gather (DCN v1, CROSS): x_{l+1} = x0 (x_l . w_l) + b_l + x_l keeps
// every x_l in span{x0, b_0 + .. + b_{l-1}}: x_l = alpha_l x0 + beta_l with
// alpha_0 = 1, beta_0 = 0, so
//   s_l = x_l . w_l = alpha_l (x0 . w_l) + c_l,   c_l = beta_l . w_l
//   alpha_{l+1} = alpha_l + s_l,  beta_{l+1} = beta_l + b_l
//   cross logit = x_L . head_w = alpha_L (x0 . head_w) + c_L
// with the c_l precomputed once per weight set (models/ctr.py DCN). The whole
// cross network of a row is L + 1 dot products of x0 - which this wave holds
// in registers - with weight rows staged in LDS, and L + 1 scalar steps: no
// x0 re-read, no per-row weight traffic from L2 (round 2's separate cross
// kernel read 66 KB of fp32 weights per row, ~1.1 GB per 16384-row step).
template <int D, typename IdT, bool ARENA, int R, bool CROSS = false>
__global__ void __launch_bounds__(256) embed_pipe_kernel(EmbedArgs a, uint64_t magic) {
  constexpr int LPR = D / 8;          // lanes per table row (16 B each)
  constexpr int FPI = kWave / LPR;    // fields per wave-wide load
  constexpr int MAXG = kWave / FPI;   // load instructions per row
  const bf16* __restrict__ table = static_cast<const bf16*>(a.table);
  const int F = a.F, B = a.B;
  extern __shared__ float4 s_cross4[];  // CROSS: [cross_n][F * D] fp32
  const float* s_cross = reinterpret_cast<const float*>(s_cross4);
  const int xd = F * D;
  if constexpr (CROSS) {
    const int n4 = a.cross_n * xd / 4;
    for (int i = threadIdx.x; i < n4; i += blockDim.x) s_cross4[i] = reinterpret_cast<const float4*>(a.cross_w)[i];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int nwaves = gridDim.x * (blockDim.x >> 6);
  // this wave's rows: b0 + k * nwaves; each iteration has R of them in flight
  const int b0 = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int sub = lane / LPR, dl = (lane % LPR) * 8;
  const bool fl_ok = lane < F;
  const int64_t m_f = (fl_ok && a.modulo_f) ? a.modulo_f[lane] : a.modulo;
  const int64_t off_f = (fl_ok && a.offset_f) ? a.offset_f[lane] : 0;
  const int64_t lo_f = (fl_ok && a.shard_lo_f) ? a.shard_lo_f[lane] : 0;
  const int64_t n_f = (fl_ok && a.shard_lo_f) ? a.shard_n_f[lane] : 0;

  // stage 1: lane f's raw id / weight of row r
  auto fetch = [&](int r, int64_t& id, float& w) {
    id = 0;
    w = 0.f;
    if (!fl_ok || r >= B) return;
    id = int64_t(static_cast<const IdT*>(a.ids)[int64_t(r) * a.ids_ld + lane]);
    w = load_weight(a, int64_t(r) * a.wts_ld + lane);
  };
  // Arena rows: stage 0 = the row's descriptor (offsets of its ids / weights),
  // loaded ONE ROW AHEAD of stage 1, so each row's id fetch is a single round
  // trip instead of the header -> descriptor -> ids chain (3 dependent loads
  // per row; the arena header is read once per wave). Served DeepFM step,
  // rocprofv3: 51.6 -> 49.9 us median per 16,384-row gather - the chain was
  // mostly hidden already; the gather is bound by table-row misses once the
  // step's GEMMs have cycled the caches (38 us back to back in isolation).
  // Padding rows past the arena's row count (no request): id 0, weight 0.
  const uint8_t* a_payload = nullptr;
  const int2* a_desc = nullptr;
  int64_t a_rows = 0;
  int a_wcols = kArenaAllWeights, a_idb = 4;
  if constexpr (ARENA) {
    const uint8_t* arena = static_cast<const uint8_t*>(a.arena);
    a_rows = *reinterpret_cast<const int64_t*>(arena + 8);
    a_wcols = arena_narrow_wcols(arena);
    a_idb = arena_narrow_idb(arena);
    a_payload = arena + kArenaPayloadOff;
    a_desc = reinterpret_cast<const int2*>(a_payload + *reinterpret_cast<const int64_t*>(arena + 16));
  }
  auto desc = [&](int r, int2& d, bool& ok) {
    ok = fl_ok && r < B && r < a_rows;
    d = ok ? a_desc[r] : int2{0, 0};
  };
  auto fetch_desc = [&](const int2& d, bool ok, int64_t& id, float& w) {
    id = 0;
    w = 0.f;
    if (!ok) return;
    const ArenaRow ar = arena_row_at(a_payload, d, a_wcols, a_idb);
    arena_feature(ar, lane, id, w);
  };
  // stage 2: hash -> table row (clamped), weight (0 for rows another shard owns)
  auto resolve = [&](int64_t id, float w_in, int64_t& row, float& w) {
    row = 0;
    w = 0.f;
    if (!fl_ok) return;
    int64_t g = magic ? hash_row_magic(id, m_f, magic) : hash_row(id, m_f);
    bool own = true;
    if (a.shard_lo_f) {
      g -= lo_f;
      own = g >= 0 && g < n_f;
      g = own ? g : 0;
    }
    row = off_f + g;
    row = row < 0 ? 0 : (row >= a.V ? a.V - 1 : row);  // memory safety whatever the tables say
    w = own ? w_in : 0.f;
  };

  int64_t id_n[R];
  float w_n[R];
  int2 d_n[R];
  bool dv_n[R];
  if constexpr (ARENA) {
#pragma unroll
    for (int k = 0; k < R; ++k) desc(b0 + k * nwaves, d_n[k], dv_n[k]);
#pragma unroll
    for (int k = 0; k < R; ++k) fetch_desc(d_n[k], dv_n[k], id_n[k], w_n[k]);
#pragma unroll
    for (int k = 0; k < R; ++k) desc(b0 + (R + k) * nwaves, d_n[k], dv_n[k]);
  } else {
#pragma unroll
    for (int k = 0; k < R; ++k) fetch(b0 + k * nwaves, id_n[k], w_n[k]);
  }
  for (int b = b0; b < B; b += R * nwaves) {
    // stage 3: every table row of these R candidates in flight, then the next
    // R rows' ids / weights behind them
    bf16x8 v[R][MAXG];
    float wf[R][MAXG], lin_w[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      int64_t row;
      float w;
      resolve(id_n[k], w_n[k], row, w);
#pragma unroll
      for (int g = 0; g < MAXG; ++g) {
        const int f = g * FPI + sub;
        const int64_t r = __shfl(row, f, 64);
        wf[k][g] = __shfl(w, f, 64);
        if (f < F && b + k * nwaves < B) {
          v[k][g] = *reinterpret_cast<const bf16x8*>(table + r * D + dl);
        } else {
          v[k][g] = bf16x8{};
          wf[k][g] = 0.f;
        }
      }
      lin_w[k] = (a.lin && fl_ok) ? a.lin[row] * w : 0.f;
    }
    if constexpr (ARENA) {
      // rows b + R*nwaves.. from the descriptors loaded last iteration, then
      // the descriptors one row further ahead
#pragma unroll
      for (int k = 0; k < R; ++k) fetch_desc(d_n[k], dv_n[k], id_n[k], w_n[k]);
#pragma unroll
      for (int k = 0; k < R; ++k) desc(b + (2 * R + k) * nwaves, d_n[k], dv_n[k]);
    } else {
#pragma unroll
      for (int k = 0; k < R; ++k) fetch(b + (R + k) * nwaves, id_n[k], w_n[k]);
    }

    // stage 4: scale, store x, FM terms
    bf16* __restrict__ out_x = static_cast<bf16*>(a.out_x);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int bk = b + k * nwaves;
      if (bk >= B) break;
      float s[8], q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
      float dots[kCrossMax];
#pragma unroll
      for (int l = 0; l < kCrossMax; ++l) dots[l] = 0.f;
      float amax = 0.f;
      bf16x8 ox[MAXG];
#pragma unroll
      for (int g = 0; g < MAXG; ++g) {
        const int f = g * FPI + sub;
        ox[g] = bf16x8{};
        if (f < F) {
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float e = bf2f(v[k][g][j]) * wf[k][g];
            s[j] += e;
            q[j] += e * e;
            o[j] = f2bf(e);
            amax = fmaxf(amax, fabsf(bf2f(o[j])));
          }
          if constexpr (CROSS) {  // x0 (as stored: bf16) . w_l for every weight row
#pragma unroll
            for (int l = 0; l < kCrossMax; ++l) {
              if (l < a.cross_n) {
                const float4* wr = reinterpret_cast<const float4*>(s_cross + l * xd + f * D + dl);
                const float4 w0 = wr[0], w1 = wr[1];
                dots[l] += bf2f(o[0]) * w0.x + bf2f(o[1]) * w0.y + bf2f(o[2]) * w0.z + bf2f(o[3]) * w0.w +
                           bf2f(o[4]) * w1.x + bf2f(o[5]) * w1.y + bf2f(o[6]) * w1.z + bf2f(o[7]) * w1.w;
              }
            }
          }
          ox[g] = o;
          if (out_x) *reinterpret_cast<bf16x8*>(out_x + int64_t(bk) * a.x_ld + int64_t(f) * D + dl) = o;
        }
      }
      if (a.out_q) {  // wave-uniform: the whole row is in this wave's registers
        uint8_t* qrow = static_cast<uint8_t*>(a.out_q) + int64_t(bk) * a.q_ld;
        amax = wave_max(amax);
        const float sc = amax > 0.f ? amax / 448.f : 1.f;
        const float inv = 1.f / sc;
        if (lane == 0) a.out_qs[bk] = sc;
#pragma unroll
        for (int g = 0; g < MAXG; ++g) {
          const int f = g * FPI + sub;
          if (f < F) {
            int lo = 0, hi = 0;
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(ox[g][0]) * inv, bf2f(ox[g][1]) * inv, lo, false);
            lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(ox[g][2]) * inv, bf2f(ox[g][3]) * inv, lo, true);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(ox[g][4]) * inv, bf2f(ox[g][5]) * inv, hi, false);
            hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(ox[g][6]) * inv, bf2f(ox[g][7]) * inv, hi, true);
            *reinterpret_cast<int2*>(qrow + int64_t(f) * D + dl) = make_int2(lo, hi);
          }
        }
        for (int64_t c = int64_t(F) * D / 8 + lane; c < a.q_ld / 8; c += kWave)
          *reinterpret_cast<int2*>(qrow + c * 8) = make_int2(0, 0);
      }
      if constexpr (CROSS) {
#pragma unroll
        for (int l = 0; l < kCrossMax; ++l)
          if (l < a.cross_n) dots[l] = wave_sum(dots[l]);
        if (lane == 0) {
          const int L = a.cross_n - 1;
          float alpha = 1.f;
          for (int l = 0; l < L; ++l) alpha += alpha * dots[l] + a.cross_c[l];  // alpha_{l+1} = alpha_l + s_l
          a.out_fm[bk] = alpha * dots[L] + a.cross_c[L];
        }
      } else if (a.out_fm) {
        const float logit = fm_row_logit<LPR>(s, q, lin_w[k], a.fm2 != 0, lane);
        if (lane == 0) a.out_fm[bk] = a.bias + logit;
      }
    }
  }
}

// ---------------------------------------------------------------- K1 front half (gather-GEMM path)
// For the fused gather-GEMM (gemm.hip gemm_gather_kernel): row b's ids and
// weights (request arena or id / weight rows) -> clamped table rows and
// weights, written FIELD-MAJOR - rows_t[f][b], wts_t[f][b], b < Mp (B rounded
// up to 256) - so the GEMM stages one K tile's 256 candidates with a single
// 4-byte LDS-DMA per lane; plus the first-order FM term
//   part0[b] = bias + sum_f lin[row(b, f)] * w(b, f).
// Rows b in [B, Mp): row 0, weight 0 (they contribute nothing).
// Block = 256 threads over 16 candidates (1024 blocks at 16384 rows: the
// kernel is three dependent round trips - descriptor, id / weight, lin - so
// it wants many waves in flight; 64-row blocks ran 21 us in the served step).
// Item i = t + 256k is (row i / F, field i % F): consecutive lanes read
// consecutive fields of one row, and a thread issues all its items' loads
// before using any. An LDS transpose then writes each field's 16 rows as one
// 64-byte store.
template <typename IdT, bool ARENA>
__global__ void __launch_bounds__(256) embed_resolve_kernel(EmbedArgs a, uint64_t magic, int32_t* __restrict__ rows_t,
                                                           float* __restrict__ wts_t, float* __restrict__ part0,
                                                           int64_t Mp) {
  constexpr int RB = 16, KMAX = (kWave * RB) / 256;  // items per thread for F <= 64
  // field stride RB + 1: the transposing stores (consecutive lanes =
  // consecutive fields) hit 64 distinct banks instead of 4
  constexpr int RS = RB + 1;
  __shared__ int32_t s_row[kWave * RS];
  __shared__ float s_w[kWave * RS];
  __shared__ float s_lin[kWave * RS];
  __shared__ int2 s_desc[RB];
  const int F = a.F, t = threadIdx.x, n = F * RB;
  const int b0 = blockIdx.x * RB;
  const uint8_t* payload = nullptr;
  int64_t a_rows = 0;
  int a_wcols = kArenaAllWeights, a_idb = 4;
  if constexpr (ARENA) {
    const uint8_t* arena = static_cast<const uint8_t*>(a.arena);
    a_rows = *reinterpret_cast<const int64_t*>(arena + 8);
    a_wcols = arena_narrow_wcols(arena);
    a_idb = arena_narrow_idb(arena);
    payload = arena + kArenaPayloadOff;
    if (t < RB) {
      const int b = b0 + t;
      const int2* desc = reinterpret_cast<const int2*>(payload + *reinterpret_cast<const int64_t*>(arena + 16));
      s_desc[t] = (b < a.B && b < a_rows) ? desc[b] : int2{0, 0};
    }
    __syncthreads();
  }
  int64_t id[KMAX];
  float w[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int i = t + 256 * k;
    id[k] = 0;
    w[k] = 0.f;
    if (i >= n) continue;
    const int r = i / F, f = i - r * F, b = b0 + r;
    if constexpr (ARENA) {
      if (b < a.B && b < a_rows) {
        const int2 d = s_desc[r];
        const ArenaRow ar = arena_row_at(payload, d, a_wcols, a_idb);
        arena_feature(ar, f, id[k], w[k]);
      }
    } else if (b < a.B) {
      id[k] = int64_t(static_cast<const IdT*>(a.ids)[int64_t(b) * a.ids_ld + f]);
      w[k] = load_weight(a, int64_t(b) * a.wts_ld + f);
    }
  }
  int32_t row[KMAX];
  float lin[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    int64_t g = magic ? hash_row_magic(id[k], a.modulo, magic) : hash_row(id[k], a.modulo);
    g = g < 0 ? 0 : (g >= a.V ? a.V - 1 : g);  // memory safety whatever the ids say
    row[k] = int32_t(g);
    lin[k] = (a.lin && t + 256 * k < n) ? a.lin[g] * w[k] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int i = t + 256 * k;
    if (i >= n) continue;
    const int r = i / F, f = i - r * F;
    s_row[f * RS + r] = row[k];
    s_w[f * RS + r] = w[k];
    s_lin[f * RS + r] = lin[k];
  }
  __syncthreads();
  for (int i = t; i < n; i += 256) {
    const int f = i / RB, r = i % RB;
    rows_t[int64_t(f) * Mp + b0 + r] = s_row[f * RS + r];
    wts_t[int64_t(f) * Mp + b0 + r] = s_w[f * RS + r];
  }
  if (t < RB) {
    float s = a.bias;
    for (int f = 0; f < F; ++f) s += s_lin[f * RS + t];
    part0[b0 + t] = s;
  }
}

// ---------------------------------------------------------------- K1b
// Sum-pooled embedding bag: out[b, :] = sum_{i in [off[b], off[b+1])} w_i * T[idx_i, :]
// One wave per bag; each lane owns 8 dims of up to D=512 (LPR<=64 lanes).
template <int D, typename IdT>
__global__ void __launch_bounds__(256) bag_kernel(const bf16* __restrict__ table, const IdT* __restrict__ idx,
                                                  const int64_t* __restrict__ offsets, const float* __restrict__ psw,
                                                  int nbags, int64_t nnz, int64_t modulo, int mean, float* __restrict__ out_f32,
                                                  bf16* __restrict__ out_bf16, int64_t out_stride) {
  constexpr int LPR = D / 8;
  constexpr int BPW = kWave / LPR;  // index slots per wave pass
  const int lane = threadIdx.x & 63;
  const int bag = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (bag >= nbags) return;
  const int sub = lane / LPR, dl = (lane % LPR) * 8;
  // clamp the CSR range so a malformed request can never read out of bounds
  const int64_t beg = min(max(offsets[bag], int64_t(0)), nnz);
  const int64_t end = min(max(offsets[bag + 1], beg), nnz);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int64_t i = beg + sub; i < end; i += BPW) {
    const int64_t r = hash_row(int64_t(idx[i]), modulo);
    const float w = psw ? psw[i] : 1.f;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(table + r * D + dl);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]) * w;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int o = LPR; o < kWave; o <<= 1) acc[j] += __shfl_xor(acc[j], o, 64);
  if (sub != 0) return;
  const float sc = (mean && end > beg) ? 1.f / float(end - beg) : 1.f;
  if (out_f32) {
    float4* p = reinterpret_cast<float4*>(out_f32 + int64_t(bag) * out_stride + dl);
    p[0] = make_float4(acc[0] * sc, acc[1] * sc, acc[2] * sc, acc[3] * sc);
    p[1] = make_float4(acc[4] * sc, acc[5] * sc, acc[6] * sc, acc[7] * sc);
  } else {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] * sc);
    *reinterpret_cast<bf16x8*>(out_bf16 + int64_t(bag) * out_stride + dl) = o;
  }
}


// ---------------------------------------------------------------- K1b routing
// Embedding model parallelism (parallel/embedding_sharding.py): the int32 row
// every (candidate b, owned-table slot) pair looks up on the table's owner,
// grouped by owner so ONE all-to-all hands each rank exactly its rows:
//   out[((s*B + b)*tm + j)*hot + h] = off[s*tm + j] + (id(b, col[s*tm + j] + h) mod mod[s*tm + j])
// s = owner rank, j = its j-th owned table (pad slots point at row off + 0).
__global__ void __launch_bounds__(256) shard_route_kernel(RouteArgs a) {
  // element i = ((s * B + b) * tm + j) * hot + h: owner s, candidate b, owned
  // table slot j, id h of the slot's bag; the slot's ids are columns
  // col[s tm + j] .. + hot - 1 of the row (one-hot: hot = 1)
  const int64_t n = int64_t(a.W) * a.B * a.tm * a.hot;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const int h = int(i % a.hot);
    const int64_t q = i / a.hot;
    const int j = int(q % a.tm);
    const int64_t sb = q / a.tm;
    const int b = int(sb % a.B), s = int(sb / a.B);
    const int slot = s * a.tm + j;
    const int c = min(max(a.col[slot] + h, 0), a.F - 1);
    int64_t id = 0;
    float w = 0.f;
    if (a.arena) {  // K0 fused: the id (and weight) straight from the request bytes
      const ArenaRow ar = arena_row(a.arena, kArenaPayloadOff, b);
      if (ar.ids) arena_feature(ar, c, id, w);
    } else {
      id = a.ids64 ? static_cast<const int64_t*>(a.ids)[int64_t(b) * a.ld + c]
                   : int64_t(static_cast<const int32_t*>(a.ids)[int64_t(b) * a.ld + c]);
      w = a.wts ? a.wts[int64_t(b) * a.wts_ld + c] : 1.f;
    }
    a.out[i] = int32_t(a.off[slot] + hash_row(id, a.mod[slot]));
    if (a.out_w) a.out_w[i] = w;
  }
}

}  // namespace kern

// ---------------------------------------------------------------- launchers
using namespace kern;

hipError_t launch_embed_resolve(const EmbedArgs& a, int32_t* rows_t, float* wts_t, float* part0, int64_t Mp,
                                hipStream_t st) {
  if (a.F < 1 || a.F > kWave || a.modulo <= 0 || a.modulo_f || a.shard_lo_f || Mp % 256 != 0 || Mp < a.B ||
      a.V < 1 || a.V > (int64_t(1) << 31) || !rows_t || !wts_t || !part0)
    return hipErrorInvalidValue;
  if (Mp == 0) return hipSuccess;
  const uint64_t magic = a.modulo < (int64_t(1) << 32) ? ~uint64_t(0) / uint64_t(a.modulo) : 0;
  dim3 grid(unsigned(Mp / 16)), block(256);
  if (a.arena)
    hipLaunchKernelGGL((embed_resolve_kernel<int64_t, true>), grid, block, 0, st, a, magic, rows_t, wts_t, part0, Mp);
  else if (a.ids64)
    hipLaunchKernelGGL((embed_resolve_kernel<int64_t, false>), grid, block, 0, st, a, magic, rows_t, wts_t, part0, Mp);
  else
    hipLaunchKernelGGL((embed_resolve_kernel<int32_t, false>), grid, block, 0, st, a, magic, rows_t, wts_t, part0, Mp);
  return hipGetLastError();
}

hipError_t launch_pack_ids(const void* ids, bool ids64, int32_t* out, int64_t n, int F, const int64_t* modulo_f,
                           const int64_t* offset_f, int64_t modulo, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const int blocks = int(std::min<int64_t>((n + 255) / 256, 2048));
  if (ids64)
    hipLaunchKernelGGL(pack_ids_kernel<int64_t>, dim3(blocks), dim3(256), 0, st, static_cast<const int64_t*>(ids),
                       out, n, F, modulo_f, offset_f, modulo);
  else
    hipLaunchKernelGGL(pack_ids_kernel<int32_t>, dim3(blocks), dim3(256), 0, st, static_cast<const int32_t*>(ids),
                       out, n, F, modulo_f, offset_f, modulo);
  return hipGetLastError();
}

hipError_t launch_shard_route(const RouteArgs& a, hipStream_t st) {
  const int64_t n = int64_t(a.W) * a.B * a.tm * a.hot;
  if (n == 0) return hipSuccess;
  if (a.F < 1 || a.hot < 1 || !a.out || (!a.ids && !a.arena)) return hipErrorInvalidValue;
  const int blocks = int(std::min<int64_t>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(shard_route_kernel, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

// Pipelined K1 grid: at most g_embed_waves waves, each walking rows with a
// stride, g_embed_rows rows in flight per wave (set_embed_wave_cap: tuning
// sweeps and tests; waves = 0 selects the one-row-per-wave kernel).
static int g_embed_waves = 4096;
static int g_embed_rows = 1;

void set_embed_wave_cap(int waves, int rows_in_flight) {
  g_embed_waves = waves < 0 ? 0 : waves;
  g_embed_rows = rows_in_flight >= 2 ? 2 : 1;
}

template <int D, int R>
static void embed_pipe_dispatch(const EmbedArgs& a, dim3 grid, dim3 block, uint64_t magic, hipStream_t st) {
  if (a.cross_n > 0) {  // DCN v1: the cross network rides on the gather (weights in LDS)
    const size_t lds = size_t(a.cross_n) * a.F * D * sizeof(float);
    if (a.arena) hipLaunchKernelGGL((embed_pipe_kernel<D, int64_t, true, R, true>), grid, block, lds, st, a, magic);
    else if (a.ids64) hipLaunchKernelGGL((embed_pipe_kernel<D, int64_t, false, R, true>), grid, block, lds, st, a, magic);
    else hipLaunchKernelGGL((embed_pipe_kernel<D, int32_t, false, R, true>), grid, block, lds, st, a, magic);
    return;
  }
  if (a.arena) hipLaunchKernelGGL((embed_pipe_kernel<D, int64_t, true, R>), grid, block, 0, st, a, magic);
  else if (a.ids64) hipLaunchKernelGGL((embed_pipe_kernel<D, int64_t, false, R>), grid, block, 0, st, a, magic);
  else hipLaunchKernelGGL((embed_pipe_kernel<D, int32_t, false, R>), grid, block, 0, st, a, magic);
}

template <int D>
static void embed_dispatch(const EmbedArgs& a, hipStream_t st) {
  const int rows_per_block = 4;
  if (a.out_q && !(a.F <= kWave && g_embed_waves > 0)) return;  // launch_embed rejects it first
  if (a.F <= kWave && g_embed_waves > 0) {
    const int waves = std::min((a.B + g_embed_rows - 1) / g_embed_rows, std::max(g_embed_waves, rows_per_block));
    dim3 grid((waves + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
    const uint64_t magic = (!a.modulo_f && a.modulo > 0 && a.modulo < (int64_t(1) << 32))
                               ? ~uint64_t(0) / uint64_t(a.modulo) : 0;
    if (g_embed_rows == 2) embed_pipe_dispatch<D, 2>(a, grid, block, magic, st);
    else embed_pipe_dispatch<D, 1>(a, grid, block, magic, st);
    return;
  }
  dim3 grid((a.B + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
  if (a.arena) hipLaunchKernelGGL((embed_kernel<D, int64_t, true>), grid, block, 0, st, a);
  else if (a.ids64) hipLaunchKernelGGL((embed_kernel<D, int64_t, false>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((embed_kernel<D, int32_t, false>), grid, block, 0, st, a);
}

hipError_t launch_embed(const EmbedArgs& a, hipStream_t st) {
  if (a.B == 0) return hipSuccess;
  // cross: pipelined kernel only, weights fit the LDS, out_fm receives the logit
  if (a.cross_n > 0 &&
      (a.F > kWave || g_embed_waves <= 0 || a.cross_n > kCrossMax || !a.cross_w || !a.cross_c || !a.out_fm ||
       (int64_t(a.F) * a.D) % 4 != 0 || int64_t(a.cross_n) * a.F * a.D * 4 > 160 * 1024))
    return hipErrorInvalidValue;
  // fp8 x: pipelined kernel only (F <= 64), whole 8-byte chunks, room for F*D columns
  if (a.out_q && (a.F > kWave || g_embed_waves <= 0 || !a.out_qs || a.q_ld < int64_t(a.F) * a.D || a.q_ld % 8))
    return hipErrorInvalidValue;
  switch (a.D) {
    case 8: embed_dispatch<8>(a, st); break;
    case 16: embed_dispatch<16>(a, st); break;
    case 32: embed_dispatch<32>(a, st); break;
    case 64: embed_dispatch<64>(a, st); break;
    case 128: embed_dispatch<128>(a, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int D>
static void bag_dispatch(const bf16* table, const void* idx, bool idx64, const int64_t* offsets, const float* psw,
                         int nbags, int64_t nnz, int64_t modulo, int mean, float* of, bf16* ob, int64_t stride, hipStream_t st) {
  dim3 grid((nbags + 3) / 4), block(256);
  if (idx64)
    hipLaunchKernelGGL((bag_kernel<D, int64_t>), grid, block, 0, st, table, static_cast<const int64_t*>(idx), offsets,
                       psw, nbags, nnz, modulo, mean, of, ob, stride);
  else
    hipLaunchKernelGGL((bag_kernel<D, int32_t>), grid, block, 0, st, table, static_cast<const int32_t*>(idx), offsets,
                       psw, nbags, nnz, modulo, mean, of, ob, stride);
}

hipError_t launch_embedding_bag(const void* table, const void* idx, bool idx64, const int64_t* offsets,
                                const float* psw, int nbags, int64_t nnz, int D, int64_t modulo, bool mean, float* out_f32,
                                void* out_bf16, int64_t out_stride, hipStream_t st) {
  if (nbags == 0) return hipSuccess;
  const bf16* t = static_cast<const bf16*>(table);
  bf16* ob = static_cast<bf16*>(out_bf16);
  switch (D) {
    case 8: bag_dispatch<8>(t, idx, idx64, offsets, psw, nbags, nnz, modulo, mean, out_f32, ob, out_stride, st); break;
    case 16: bag_dispatch<16>(t, idx, idx64, offsets, psw, nbags, nnz, modulo, mean, out_f32, ob, out_stride, st); break;
    case 32: bag_dispatch<32>(t, idx, idx64, offsets, psw, nbags, nnz, modulo, mean, out_f32, ob, out_stride, st); break;
    case 64: bag_dispatch<64>(t, idx, idx64, offsets, psw, nbags, nnz, modulo, mean, out_f32, ob, out_stride, st); break;
    case 128: bag_dispatch<128>(t, idx, idx64, offsets, psw, nbags, nnz, modulo, mean, out_f32, ob, out_stride, st); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dtfs

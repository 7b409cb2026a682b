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
        id = arow.ids ? int64_t(load_u64_unaligned(arow.ids + 8 * fl)) : 0;
        w_in = arow.ids ? __uint_as_float(load_u32_unaligned(arow.wts + 4 * fl)) : 0.f;
      } else {
        id = int64_t(ids[int64_t(b) * a.ids_ld + fl]);
        w_in = a.wts ? a.wts[int64_t(b) * a.wts_ld + fl] : 1.f;
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
  float fm = 0.f;
  if (a.fm2) {
    // sum over fields: lanes with the same (lane % LPR) own the same dims
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int o = LPR; o < kWave; o <<= 1) {
        s[j] += __shfl_xor(s[j], o, 64);
        q[j] += __shfl_xor(q[j], o, 64);
      }
    }
    float part = 0.f;
    if (lane < LPR) {
#pragma unroll
      for (int j = 0; j < 8; ++j) part += s[j] * s[j] - q[j];
    }
    fm = 0.5f * wave_sum(part);
  }
  const float fo = a.lin ? wave_sum(first) : 0.f;
  if (lane == 0) a.out_fm[b] = a.bias + fo + fm;
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

}  // namespace kern

// ---------------------------------------------------------------- launchers
using namespace kern;

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

template <int D>
static void embed_dispatch(const EmbedArgs& a, hipStream_t st) {
  const int rows_per_block = 4;
  dim3 grid((a.B + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
  if (a.arena) hipLaunchKernelGGL((embed_kernel<D, int64_t, true>), grid, block, 0, st, a);
  else if (a.ids64) hipLaunchKernelGGL((embed_kernel<D, int64_t, false>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((embed_kernel<D, int32_t, false>), grid, block, 0, st, a);
}

hipError_t launch_embed(const EmbedArgs& a, hipStream_t st) {
  if (a.B == 0) return hipSuccess;
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

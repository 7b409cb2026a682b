// Host-side launch entry points of the gfx950 kernels. Raw pointers + a HIP
// stream only: no torch types, so the kernels compile with plain hipcc and the
// launchers are capturable into HIP graphs (no allocation, no sync inside).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtfs {

// K0: out[i] = offset[f] + ((ids[i] % m_f) + m_f) % m_f, f = i % F.
hipError_t launch_pack_ids(const void* ids, bool ids64, int32_t* out, int64_t n, int F, const int64_t* modulo_f,
                           const int64_t* offset_f, int64_t modulo, hipStream_t st);

// K1b routing: out[(s*B + b)*tm + j] = off[s*tm+j] + (ids[b*ld + col[s*tm+j]] mod mod[s*tm+j])
// (int32 rows grouped by owner rank for the embedding all-to-all); col is
// clamped into [0, F).
// K1b routing (embedding model parallelism): table rows (and weights) of
// every candidate grouped by owner rank, out[s][b][j][h] = off[s tm + j] +
// (id(b, col[s tm + j] + h) mod mod[s tm + j]); ids from an [B, F] row view or
// straight from a device request arena.
struct RouteArgs {
  const void* ids = nullptr;
  bool ids64 = true;
  int64_t ld = 0;
  const uint8_t* arena = nullptr;  // instead of ids (+ wts)
  const float* wts = nullptr;      // optional per-id weights (multi-hot bags)
  int64_t wts_ld = 0;
  int B = 0, F = 0, W = 1, tm = 1, hot = 1;
  const int32_t* col = nullptr;
  const int64_t* mod = nullptr;
  const int64_t* off = nullptr;
  int32_t* out = nullptr;   // [W, B, tm, hot]
  float* out_w = nullptr;   // optional, same shape
};
hipError_t launch_shard_route(const RouteArgs& a, hipStream_t st);

// K1: weighted gather (+ first/second-order FM). out_x bf16 [B, F*D] and/or out_fm fp32 [B].
struct EmbedArgs {
  const void* table = nullptr;     // bf16 [V, D]
  const float* lin = nullptr;      // fp32 [V] first-order weights (optional)
  const void* ids = nullptr;       // int32/int64 [B, ids_ld] (first F used)
  bool ids64 = true;
  int64_t ids_ld = 0;
  const void* wts = nullptr;       // fp32 (or bf16 with wts16) [B, wts_ld] (optional)
  int64_t wts_ld = 0;
  bool wts16 = false;
  int B = 0, F = 0, D = 0;
  int64_t V = 0;                   // table rows (rows are clamped into [0, V))
  int64_t modulo = 0;              // shared-table hashing
  const int64_t* modulo_f = nullptr;  // per-field tables: row = offset_f[f] + id mod modulo_f[f]
  const int64_t* offset_f = nullptr;
  // row-wise sharded tables: this process holds global rows [lo_f, lo_f + n_f)
  // of field f's table at offset_f[f]; ids hashing outside contribute zeros
  // (the partial embeddings are summed across ranks by a reduce-scatter)
  const int64_t* shard_lo_f = nullptr;
  const int64_t* shard_n_f = nullptr;
  // request arena (csrc/runtime/arena.h): when set, row b's ids / weights are
  // read straight from the raw request bytes (ids / wts above are unused) -
  // the embedding gather doubles as the ingest unpack
  const void* arena = nullptr;
  float bias = 0.f;
  void* out_x = nullptr;           // bf16 [B, x_ld]
  int64_t x_ld = 0;
  float* out_fm = nullptr;         // fp32 [B]
  int fm2 = 0;
  // fp8 copy of x for the fp8 towers (pipelined kernel, F <= 64 only): per-row
  // e4m3 of the bf16-rounded x with scale amax / 448 (quant_rows_fp8's
  // rounding), columns [F*D, q_ld) zeroed - saves a separate quant pass
  void* out_q = nullptr;           // e4m3 [B, q_ld]
  int64_t q_ld = 0;
  float* out_qs = nullptr;         // fp32 [B]
  // DCN v1 cross network inside the gather (pipelined kernel, F <= 64 only):
  // cross_w = [w_0 .. w_{L-1}, head_w] fp32 [cross_n][F*D], cross_c fp32
  // [cross_n]; out_fm[b] receives the cross half of the head logit (see
  // embedding.hip, "K3 in the gather")
  const float* cross_w = nullptr;
  const float* cross_c = nullptr;
  int cross_n = 0;                 // L + 1, at most kCrossMax
};
constexpr int kCrossMax = 8;
hipError_t launch_embed(const EmbedArgs& a, hipStream_t st);
// Pipelined K1 kernel geometry: resident-wave cap (0 = one row per wave) and
// rows in flight per wave (1 or 2).
void set_embed_wave_cap(int waves, int rows_in_flight = 1);

// Front half of K1 for the gather-GEMM (gemm_gather): shared-table rows /
// weights of B candidates, field-major rows_t / wts_t [F][Mp] (Mp = B rounded
// up to 256; padding rows: row 0, weight 0), and part0[b] = bias + the
// first-order FM term. ids / wts / arena / lin / modulo / V / B / F / bias of
// `a` are read; the outputs above replace out_x / out_fm.
hipError_t launch_embed_resolve(const EmbedArgs& a, int32_t* rows_t, float* wts_t, float* part0, int64_t Mp,
                                hipStream_t st);

// K0 ingest: request arena (header + descriptors + raw request bytes) -> packed
// rows [B, W] int64 (serving/arena.py, csrc/runtime/arena.h share the layout).
constexpr int kArenaPayloadOff = 64 + 32 * 1024;  // descriptors: up to 1024 requests
constexpr int kArenaMaxRequests = 1024;
// narrow_modulo > 0: narrow rows [int32 (id mod m) x F | fp32 weights x F | pad].
hipError_t launch_unpack_arena(const void* arena, int64_t* packed, int B, int F, int W, int max_req,
                               hipStream_t st, int64_t narrow_modulo = 0);
// Packed varint ids of a built arena -> its device-only int64 id region
// (csrc/runtime/arena.h VarintChunk); blocks loop over the chunk table.
hipError_t launch_arena_varint(void* arena, int blocks, hipStream_t st);
// Host stub of that kernel (lets a replayed step skip it when no request of
// the step has varint ids: runtime/kernel_seq.cpp).
const void* arena_varint_kernel_fn();
// H2D pulled by GPU waves from pinned host memory (16-B aligned src and dst).
hipError_t launch_pull_host(void* dst, const void* src, int64_t nbytes, int blocks, hipStream_t st);

// K1b: sum/mean embedding bag with CSR offsets [nbags+1].
hipError_t launch_embedding_bag(const void* table, const void* idx, bool idx64, const int64_t* offsets,
                                const float* psw, int nbags, int64_t nnz, int D, int64_t modulo, bool mean, float* out_f32,
                                void* out_bf16, int64_t out_stride, hipStream_t st);

// Block-scaled (OCP MX) fp8 activations on the fp8 GEMM path: e4m3 values with
// one E8M0 scale byte per 32 consecutive K elements of a row.
//   sab != nullptr : A's block scales [M][ldsab], fed to the MFMA scale operand
//   q   != nullptr : the (cross) epilogue also writes its output as e4m3 q
//                    [M][ldq] + block scales sq [M][ldsq]; columns [N, nq) of q
//                    are zero (the consumer's K padding)
struct MxIO {
  const uint8_t* sab = nullptr;
  int64_t ldsab = 0;
  uint8_t* q = nullptr;
  int64_t ldq = 0;
  uint8_t* sq = nullptr;
  int64_t ldsq = 0;
  int nq = 0;
};

// K1 fused into K4 (gemm.hip gemm_gather_kernel): C bf16 [M, N] =
// epi(sum_f bf16(w * T[row]) . W[:, 64f:64f+64]^T + bias) for a bf16 table
// with 64-wide rows (128 B), rows_t / wts_t from launch_embed_resolve, W bf16
// [N, 64F]; N % 256 == 0. fm_part (N >= 1024): row 1 of the [2][Mp] FM
// partials receives the second-order FM term.
// cross_w / cross_c / cross_n (DCN v1, with fm_part): the folded cross
// weights fp32 [cross_n][64F] + constants (EmbedArgs.cross_*, cross_n <= 4);
// fm_part's row 1 then receives the cross logit instead of the FM term.
hipError_t launch_gemm_gather(const void* table, int64_t V, const int32_t* rows_t, const float* wts_t, int64_t Mp,
                              int F, const void* W, const float* bias, void* C, int64_t ldc, float* fm_part, int M,
                              int N, int epi, hipStream_t st, const float* cross_w = nullptr,
                              const float* cross_c = nullptr, int cross_n = 0);

// The same op, one wave per SIMD (gather_gemm.hip): Wp = W in MFMA fragment
// order (ops.pack_frag32), N % 512 == 0, Mp % 128 == 0, V <= 2^25 table rows;
// no cross network.
bool gemm_gather1w_ok(int64_t Mp, int N, int F, bool cross, int64_t V);
hipError_t launch_gemm_gather1w(const void* table, int64_t V, const int32_t* rows_t, const float* wts_t, int64_t Mp,
                                int F, const void* Wp, const float* bias, void* C, int64_t ldc, float* fm_part, int M,
                                int N, int epi, hipStream_t st);

// K3b/K4: C = epi(A[M,K] . W[N,K]^T); epi: 0 none, 1 relu, 2 sigmoid, 3 cross.
hipError_t launch_gemm(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, const float* sa,
                       const float* sw, void* C, int64_t ldc, bool out_f32, const void* X0, const void* XL,
                       int64_t ldx, int M, int N, int K, int epi, bool fp8, hipStream_t st,
                       int variant = 0, const MxIO* mx = nullptr);

// K4+K6 fused: y[m] = out_act(act(A W^T + b)[m,:] . hw + hbias + extra[m]); N <= 256, bf16.
// extra_n > 1: extra holds extra_n partial logits, extra[e * extra_ld + m]
// (the gather-GEMM path's first-order + FM partitions), summed in order.
hipError_t launch_gemm_head(const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias, int act,
                            const float* hw, float hbias, const float* extra, int out_act, float* y, int M, int N,
                            int K, hipStream_t st, int extra_n = 1, int64_t extra_ld = 0);

// K4 + K4 + K6 fused MLP tail (mlp_tail.hip): h2 = act2(X W2^T + b2) (bf16, in
// LDS), y[m] = out_act(act3(h2 W3^T + b3)[m,:] . hw + hbias + sum_e extra[e][m]).
// W2p / W3p: the weights in MFMA fragment order (ops.pack_bfrag). N2 = 512,
// N3 = 256, K1 = 1024; out_act 0 none / 2 sigmoid; y device or mapped host.
hipError_t launch_mlp_tail(const void* X, int64_t ldx, int M, int K1, const void* W2p, const float* b2, int act2,
                           int N2, const void* W3p, const float* b3, int act3, int N3, const float* hw, float hbias,
                           const float* extra, int extra_n, int64_t extra_ld, int out_act, float* y, hipStream_t st);

// K1 + K2 + K4 x 3 + K6 (gather_mlp.hip): the DeepFM / Wide&Deep tower in one
// launch, the resolve pass included: a.table / V / lin / modulo / bias and the
// rows (a.arena, or a.ids + a.wts) as for launch_embed_resolve, a.B rows, a.F
// fields; y[m] = out_act(act3(act2(relu(x W1^T + b1) W2^T + b2) W3^T + b3) . hw
// + hbias + bias + sum_f lin[row] w (+ FM(m) when fm)); W1p / W2p / W3p in
// 32x32x16 fragment order (ops.pack_frag32); N1 = 1024, N2 = 512, N3 = 256,
// F <= 64, V <= 2^25.
bool gather_mlp_ok(int64_t Mp, int N1, int K1, int N2, int N3, int F, int64_t V);
hipError_t launch_gather_mlp(const EmbedArgs& a, const void* W1p, const float* b1, const void* W2p, const float* b2,
                             int act2, const void* W3p, const float* b3, int act3, const float* hw, float hbias,
                             bool fm, int out_act, float* y, hipStream_t st);

// K3: DCN-v1 cross network, all L layers fused.
hipError_t launch_cross_v1(const void* x0, int64_t ldx, int B, int d, int L, const float* w, const float* b,
                           void* out_x, int64_t ldo, const float* head_w, float* out_dot, hipStream_t st);

// K5: DLRM dot interaction (T + 1 <= 32, D = 64). Table t's vector of row b is
// emb row (b*T + t), or with a table map (emb_off / emb_stride, int64 [T])
// emb row (emb_off[t] + b*emb_stride[t]), clamped into [0, emb_rows) - the
// layout an embedding all-to-all leaves behind, read in place.
hipError_t launch_dot_interaction(const void* dense, int64_t ldd, const void* emb, int T, int B, void* out,
                                  int64_t ldo, int out_cols, hipStream_t st, const int64_t* emb_off = nullptr,
                                  const int64_t* emb_stride = nullptr, int64_t emb_rows = 0);

// DLRM dense input: y bf16 [M, K] = x[:, :n] (fp32, row stride ldx) zero padded; K % 8 == 0.
hipError_t launch_dense_pad(const float* x, int64_t ldx, int M, int n, void* y, int K, hipStream_t st);

// K6: y = act(x . w + bias + extra), act 0 none / 2 sigmoid (extra_n / extra_ld: launch_gemm_head).
hipError_t launch_head(const void* x, int64_t ldx, const float* w, float bias, const float* extra, int M, int K,
                       int act, float* out, hipStream_t st, int extra_n = 1, int64_t extra_ld = 0);

// fp8 (OCP e4m3) per-row quantisation.
// Kq >= K: output row width; columns [K, Kq) are zeroed (K padding for the
// 128-deep block-scaled fp8 MFMA). 0 = K.
hipError_t launch_quant_rows_fp8(const void* x, int64_t ldx, int M, int K, void* q, int64_t ldq, float* scale,
                                 hipStream_t st, int Kq = 0);

// K3b split: z = x0 * y + xl per row (bf16 [M, N], row stride ld), optionally
// written (z), quantised to e4m3 + per-row scale with zero K padding to Kq (q,
// scale), and/or reduced against head_w (dot[m] = z . head_w).
hipError_t launch_cross_combine(const void* y, const void* x0, const void* xl, int64_t ld, int M, int N, void* z,
                                int64_t ldz, void* q, int64_t ldq, float* scale, int Kq, const float* head_w,
                                float* dot, hipStream_t st);

// DCN-v2 cross layer in one launch (fp8 8-phase GEMM + LDS-staged cross
// epilogue): y = (A W^T) * sa * sw + b, z = bf16(x0 * bf16(y) + xl), written
// to Z and / or dotted with hw into one partial logit per 256-column tile:
// dot[tn * ldd + m], tn < ceil(N / 256). A: e4m3 [M][K] with per-row scales
// sa, K % 128 == 0; N % 8 == 0.
struct CrossGemmArgs {
  const void* A = nullptr;
  int64_t lda = 0;
  const void* W = nullptr;
  int64_t ldw = 0;
  const float* bias = nullptr;
  const float* sa = nullptr;
  const float* sw = nullptr;
  void* Z = nullptr;
  int64_t ldz = 0;
  const void* X0 = nullptr;
  const void* XL = nullptr;
  int64_t ldx = 0;
  const float* hw = nullptr;
  float* dot = nullptr;
  int64_t ldd = 0;
  int M = 0, N = 0, K = 0;
};
hipError_t launch_cross_gemm_fp8(const CrossGemmArgs& args, hipStream_t st);
// (The rejected one-wave-per-SIMD form of this layer, 128 x 512 tiles with W
// in MX fragment order, lives in tools/native/cross_gemm_1w.hip with its stamp
// study; profiles/r05_dcn_cross1w.md.)

// Peer lookup (kernels/peer_lookup.h): table-wise sharded tables read
// one-sidedly where they live. A rank's store is a list of chunks of 2^shift
// rows (separate allocations, each mapped by the peers through IPC); chunk c
// of rank r is at device address cbase[r * max_chunks + c]. Row v of table t
// (v = id mod trows[t]) is row g = toff[t] + v of rank towner[t]'s store.
// tremote[t] = 1 marks a table owned by another rank, whose rows are looked
// up in the replica cache first. cache = device int64 [5] {index (entries
// int64 [mask + 1][2] = {key, slot}, key -1 = empty; 0 = no index), unused,
// mask, rows [cap][64] bf16, cap}, read by each wave at its start (the host
// swaps indices by rewriting word 0). Candidates b with b % sample_every ==
// sample_every / 2 (all when sample_every <= 1) are counted - stats [128]:
// hits at 2i, misses at 2i + 1 (i = block % 64); when sample_every > 0,
// candidates with b % sample_every == 0 push their remote keys (t << 40 | v)
// into ring: 64 segments of ring_cap / 64 keys, segment block % 64 written at
// ring_ctr[block % 64] (int64 [64], wrapping).
struct PeerLookupArgs {
  const int64_t* cbase = nullptr;
  const int32_t* towner = nullptr;
  const int64_t* toff = nullptr;
  const int64_t* trows = nullptr;
  const int32_t* tremote = nullptr;
  int chunk_shift = 0;
  int max_chunks = 0;
  const int64_t* cache = nullptr;
  unsigned long long* stats = nullptr;
  int64_t* ring = nullptr;
  unsigned long long* ring_ctr = nullptr;
  int64_t ring_cap = 0;
  int sample_every = 0;
};

// K1 + K5: DLRM dot interaction with the one-hot gather fused in: vector t+1
// of row b is table[offset_f[t] + ids[b * ldi + t] mod modulo_f[t]] (rows
// clamped to the table); out [B][ldo] = [dense | lower triangle | zeros].
// arena (a device request arena): the ids are features id_col0 .. id_col0 +
// T - 1 of arena row b instead (ids unused). peer: the rows come through the
// peer lookup instead (table, table_rows, modulo_f, offset_f unused).
hipError_t launch_dot_interaction_gather(const void* dense, int64_t ldd, const void* table, int64_t table_rows,
                                         const void* ids, bool ids64, int64_t ldi, const int64_t* modulo_f,
                                         const int64_t* offset_f, int T, int B, void* out, int64_t ldo, int out_cols,
                                         hipStream_t st, const void* arena = nullptr, int id_col0 = 0,
                                         const PeerLookupArgs* peer = nullptr);

// K1b through the peer lookup: out[b][t] (bf16 [B][T][64]) = sum_j w(b, c) *
// row(t, id(b, c)), c = col0 + t * hot + j (ids / wts [B][F] row views, or
// the features of a device request arena row).
hipError_t launch_peer_bag(const PeerLookupArgs& p, const void* ids, bool ids64, int64_t ldi, const float* wts,
                           int64_t ldw, const void* arena, int col0, int T, int hot, int B, void* out,
                           hipStream_t st);

// Replica cache maintenance: rows[slots[i]] = row (keys[i] & (2^40 - 1)) of
// table keys[i] >> 40 (read where it lives: over xGMI for a peer's table);
// and the open-addressing index (entries [mask + 1][2] pre-filled with -1,
// mask + 1 a power of two >= 2 n) mapping keys[i] -> slots[i].
hipError_t launch_peer_cache_fill(const PeerLookupArgs& p, int T, const int64_t* keys, const int32_t* slots,
                                  int64_t n, void* rows, int64_t cap, hipStream_t st);
hipError_t launch_cache_index_build(const int64_t* keys, const int32_t* slots, int64_t n, int64_t* entries,
                                    int64_t mask, hipStream_t st);

// K4 (small) for the DLRM bottom MLP: relu(relu(relu(pad64(bf16(wts[:, :nd]))
// W1^T + b1) W2^T + b2) W3^T + b3) in one kernel (W1 [N1][64], W2 [N2][N1], W3
// [N3][N2] bf16; out bf16 [M][ldo]; arena: the weights are the first nd
// features of each request-arena row instead). Built for (N1, N2, N3) = (512, 256, 64);
// hipErrorInvalidValue for other shapes.
hipError_t launch_bottom_mlp3(const float* wts, int64_t ldw, int nd, int M, const void* W1, const float* b1, int N1,
                              const void* W2, const float* b2, int N2, const void* W3, const float* b3, int N3,
                              void* out, int64_t ldo, hipStream_t st, const void* arena = nullptr);

// K7: bitonic sort of n <= sort_max_elems() scores; first k_out of (sorted, perm).
int sort_max_elems();
hipError_t launch_sort_scores(const float* in, int n, bool descending, float* out, int64_t* perm, int k_out,
                              hipStream_t st);

}  // namespace dtfs

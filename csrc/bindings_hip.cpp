// torch bindings for the gfx950 kernels (distributed_tf_serving_amd/_hip*.so).
//
// Every entry point validates shapes, dtypes, devices and contiguity on the
// host BEFORE launching, because a hand-written kernel that indexes past its
// operands can take the whole GPU node down. Kernels run on the caller's
// current HIP stream, so they compose with torch streams and HIP-graph capture.
#include <torch/extension.h>

#include <cstring>

#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "kernels/launchers.h"
#include "comm/rccl_comm.h"
#include "live_bindings.h"
#include "runtime/numa.h"
#include "runtime/step_runner.h"

namespace {

hipStream_t cur_stream(const torch::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

void check_dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// device only: for row views whose strides the caller checks itself
void check_gpu(const torch::Tensor& t, const char* name) { TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor"); }

void check_same_dev(const torch::Tensor& a, const torch::Tensor& b, const char* name) {
  TORCH_CHECK(a.device() == b.device(), name, " must be on ", a.device());
}

const void* opt_ptr(const c10::optional<torch::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ---------------------------------------------------------------- K0
torch::Tensor pack_ids(torch::Tensor ids, int64_t modulo, c10::optional<torch::Tensor> modulo_f,
                       c10::optional<torch::Tensor> offset_f) {
  check_dev(ids, "ids");
  TORCH_CHECK(ids.dim() == 2, "ids must be [B, F]");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 || ids.scalar_type() == torch::kInt32, "ids must be int32/int64");
  const int F = int(ids.size(1));
  for (auto* o : {&modulo_f, &offset_f})
    if (o->has_value()) {
      check_dev(**o, "per-field table");
      TORCH_CHECK((*o)->scalar_type() == torch::kInt64 && (*o)->numel() == F, "per-field tables must be int64 [F]");
    }
  c10::DeviceGuard g(ids.device());
  auto out = torch::empty(ids.sizes(), ids.options().dtype(torch::kInt32));
  check_hip(dtfs::launch_pack_ids(ids.data_ptr(), ids.scalar_type() == torch::kInt64, out.data_ptr<int32_t>(),
                                  ids.numel(), F, modulo_f ? modulo_f->data_ptr<int64_t>() : nullptr,
                                  offset_f ? offset_f->data_ptr<int64_t>() : nullptr, modulo, cur_stream(ids)),
            "pack_ids");
  return out;
}

// ---------------------------------------------------------------- K1
// k_pad > 0: the gather also writes x as e4m3 [B, K rounded up to k_pad] + a
// per-row scale (the fp8 towers' first operand; replaces quant_rows_fp8(x)).
// DCN v1 cross network inside the gather (embedding.hip): weight rows
// [w_0 .. w_{L-1}, head_w] fp32 [L+1, F*D] and constants fp32 [L+1]; the
// gather's fm output becomes the cross logit.
static void embed_cross_in(dtfs::EmbedArgs& a, const torch::Tensor& table, int64_t F, int64_t D,
                           const c10::optional<torch::Tensor>& cross_w, const c10::optional<torch::Tensor>& cross_c) {
  if (!cross_w) return;
  TORCH_CHECK(cross_c.has_value(), "cross_w needs cross_c");
  check_same_dev(table, *cross_w, "cross_w");
  check_same_dev(table, *cross_c, "cross_c");
  TORCH_CHECK(cross_w->scalar_type() == torch::kFloat32 && cross_w->is_contiguous() && cross_w->dim() == 2 &&
                  cross_w->size(1) == F * D && cross_w->size(0) >= 1 && cross_w->size(0) <= dtfs::kCrossMax,
              "cross_w must be contiguous fp32 [L+1 <= 8, F*D]");
  TORCH_CHECK(cross_c->scalar_type() == torch::kFloat32 && cross_c->is_contiguous() &&
                  cross_c->numel() == cross_w->size(0),
              "cross_c must be fp32 [L+1]");
  TORCH_CHECK(F <= 64 && (F * D) % 4 == 0 && cross_w->numel() * 4 <= 160 * 1024,
              "cross in the gather: F <= 64 and the weights must fit the LDS");
  a.cross_w = cross_w->data_ptr<float>();
  a.cross_c = cross_c->data_ptr<float>();
  a.cross_n = int(cross_w->size(0));
}

static void embed_fp8_out(dtfs::EmbedArgs& a, const torch::Tensor& table, int64_t B, int64_t K, int64_t k_pad,
                          torch::Tensor& q, torch::Tensor& qs) {
  if (k_pad <= 0) return;
  TORCH_CHECK(k_pad <= 256, "k_pad must be in [0, 256]");
  const int64_t Kq = (K + k_pad - 1) / k_pad * k_pad;
  TORCH_CHECK(Kq % 16 == 0 && a.F <= 64, "fp8 x needs F <= 64 and a padded K that is a multiple of 16");
  q = torch::empty({B, Kq}, table.options().dtype(torch::kFloat8_e4m3fn));
  qs = torch::empty({B}, table.options().dtype(torch::kFloat32));
  a.out_q = q.data_ptr();
  a.q_ld = Kq;
  a.out_qs = qs.data_ptr<float>();
}

std::vector<torch::Tensor> embed(torch::Tensor table, c10::optional<torch::Tensor> lin, torch::Tensor ids,
                                 c10::optional<torch::Tensor> wts, int64_t modulo, c10::optional<torch::Tensor> modulo_f,
                                 c10::optional<torch::Tensor> offset_f, double bias, bool want_x, bool want_fm,
                                 bool fm2, c10::optional<torch::Tensor> out_x, bool validate_tables,
                                 c10::optional<torch::Tensor> shard_lo_f, c10::optional<torch::Tensor> shard_n_f,
                                 int64_t k_pad, c10::optional<torch::Tensor> cross_w,
                                 c10::optional<torch::Tensor> cross_c) {
  check_dev(table, "table");
  TORCH_CHECK(ids.is_cuda(), "ids must be a GPU tensor");
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2, "table must be bf16 [V, D]");
  TORCH_CHECK(ids.dim() == 2, "ids must be [B, F]");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 || ids.scalar_type() == torch::kInt32, "ids must be int32/int64");
  // ids / wts may be row views of a packed request buffer: unit inner stride,
  // any row stride >= F
  TORCH_CHECK(ids.stride(1) == 1 && ids.stride(0) >= ids.size(1), "ids rows must be contiguous");
  const int64_t B = ids.size(0), F = ids.size(1), D = table.size(1);
  TORCH_CHECK(D == 8 || D == 16 || D == 32 || D == 64 || D == 128, "embedding dim must be 8/16/32/64/128");
  check_same_dev(table, ids, "ids");
  const int64_t V = table.size(0);
  if (modulo_f.has_value() || offset_f.has_value()) {
    TORCH_CHECK(modulo_f.has_value() && offset_f.has_value(), "modulo_f and offset_f go together");
    for (auto* o : {&modulo_f, &offset_f}) {
      check_dev(**o, "per-field table");
      TORCH_CHECK((*o)->scalar_type() == torch::kInt64 && (*o)->numel() == F, "per-field tables must be int64 [F]");
    }
    // every (offset + row) must stay inside the table. The kernel also clamps
    // rows into [0, V), so this (syncing) host check is a debugging aid that
    // models run once at construction, not per batch.
    if (shard_lo_f.has_value() || shard_n_f.has_value()) {
      TORCH_CHECK(shard_lo_f.has_value() && shard_n_f.has_value(), "shard_lo_f and shard_n_f go together");
      for (auto* o : {&shard_lo_f, &shard_n_f}) {
        check_dev(**o, "shard range");
        TORCH_CHECK((*o)->scalar_type() == torch::kInt64 && (*o)->numel() == F, "shard ranges must be int64 [F]");
      }
    }
    auto mf = validate_tables ? modulo_f->cpu() : torch::Tensor();
    auto of = validate_tables ? offset_f->cpu() : torch::Tensor();
    auto sn = validate_tables && shard_n_f ? shard_n_f->cpu() : torch::Tensor();
    for (int64_t f = 0; validate_tables && f < F; ++f) {
      TORCH_CHECK(mf.data_ptr<int64_t>()[f] > 0, "per-field modulo must be > 0");
      // a row-wise shard holds n_f rows at offset_f; a whole table holds modulo_f rows
      const int64_t held = sn.defined() ? sn.data_ptr<int64_t>()[f] : mf.data_ptr<int64_t>()[f];
      TORCH_CHECK(of.data_ptr<int64_t>()[f] >= 0 && held >= 0 && of.data_ptr<int64_t>()[f] + held <= V,
                  "field ", f, " rows exceed the table");
    }
  } else {
    TORCH_CHECK(!shard_lo_f.has_value() && !shard_n_f.has_value(), "row shards need per-field tables");
    TORCH_CHECK(modulo > 0 && modulo <= V, "modulo must be in (0, table rows]: ids are hashed onto rows");
  }
  if (wts) {
    TORCH_CHECK(wts->is_cuda() && (wts->scalar_type() == torch::kFloat32 || wts->scalar_type() == torch::kBFloat16) &&
                    wts->dim() == 2 && wts->size(0) == B && wts->size(1) == F && wts->stride(1) == 1 &&
                    wts->stride(0) >= F,
                "wts must be fp32 / bf16 [B, F] with contiguous rows");
    check_same_dev(table, *wts, "wts");
  }
  if (lin) {
    check_dev(*lin, "lin");
    TORCH_CHECK(lin->scalar_type() == torch::kFloat32 && lin->numel() == V, "lin must be fp32 [V]");
  }
  c10::DeviceGuard g(ids.device());
  torch::Tensor x, fm;
  if (want_x) {
    if (out_x) {
      check_dev(*out_x, "out_x");
      TORCH_CHECK(out_x->scalar_type() == torch::kBFloat16 && out_x->numel() == B * F * D, "out_x must be bf16 [B, F*D]");
      x = *out_x;
    } else {
      x = torch::empty({B, F * D}, table.options());
    }
  }
  if (want_fm) fm = torch::empty({B}, table.options().dtype(torch::kFloat32));
  dtfs::EmbedArgs a;
  a.table = table.data_ptr();
  a.lin = lin ? lin->data_ptr<float>() : nullptr;
  a.ids = ids.data_ptr();
  a.ids64 = ids.scalar_type() == torch::kInt64;
  a.ids_ld = ids.stride(0);
  a.wts = wts ? wts->data_ptr() : nullptr;
  a.wts16 = wts && wts->scalar_type() == torch::kBFloat16;
  a.wts_ld = wts ? wts->stride(0) : 0;
  a.B = int(B);
  a.F = int(F);
  a.D = int(D);
  a.V = V;
  a.modulo = modulo;
  a.modulo_f = modulo_f ? modulo_f->data_ptr<int64_t>() : nullptr;
  a.offset_f = offset_f ? offset_f->data_ptr<int64_t>() : nullptr;
  a.shard_lo_f = shard_lo_f ? shard_lo_f->data_ptr<int64_t>() : nullptr;
  a.shard_n_f = shard_n_f ? shard_n_f->data_ptr<int64_t>() : nullptr;
  a.bias = float(bias);
  a.out_x = want_x ? x.data_ptr() : nullptr;
  a.x_ld = F * D;
  a.out_fm = want_fm ? fm.data_ptr<float>() : nullptr;
  a.fm2 = fm2 ? 1 : 0;
  torch::Tensor q, qs;
  embed_fp8_out(a, table, B, F * D, k_pad, q, qs);
  TORCH_CHECK(!cross_w || (want_fm && !modulo_f && !shard_lo_f), "cross: shared table, want_fm");
  embed_cross_in(a, table, F, D, cross_w, cross_c);
  check_hip(dtfs::launch_embed(a, cur_stream(ids)), "embed");
  return {x, fm, q, qs};
}

// K0+K1(+K2): the gather reads ids / weights straight from a device request
// arena (csrc/runtime/arena.h) - no separate unpack kernel, no packed rows.
std::vector<torch::Tensor> embed_arena(torch::Tensor table, c10::optional<torch::Tensor> lin, torch::Tensor arena,
                                       int64_t B, int64_t F, int64_t modulo, double bias, bool want_x, bool want_fm,
                                       bool fm2, c10::optional<torch::Tensor> out_x, int64_t k_pad,
                                       c10::optional<torch::Tensor> cross_w, c10::optional<torch::Tensor> cross_c) {
  check_dev(table, "table");
  check_dev(arena, "arena");
  check_same_dev(table, arena, "arena");
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2, "table must be bf16 [V, D]");
  TORCH_CHECK(arena.scalar_type() == torch::kUInt8 && arena.is_contiguous() && arena.numel() > dtfs::kArenaPayloadOff,
              "arena must be a contiguous uint8 device buffer");
  const int64_t D = table.size(1), V = table.size(0);
  TORCH_CHECK(D == 8 || D == 16 || D == 32 || D == 64 || D == 128, "embedding dim must be 8/16/32/64/128");
  TORCH_CHECK(F >= 1 && F <= 64, "arena gather handles 1..64 fields");
  TORCH_CHECK(modulo > 0 && modulo <= V, "modulo must be in (0, table rows]");
  if (lin) {
    check_dev(*lin, "lin");
    TORCH_CHECK(lin->scalar_type() == torch::kFloat32 && lin->numel() == V, "lin must be fp32 [V]");
  }
  c10::DeviceGuard g(table.device());
  torch::Tensor x, fm;
  if (want_x) {
    if (out_x) {
      check_dev(*out_x, "out_x");
      TORCH_CHECK(out_x->scalar_type() == torch::kBFloat16 && out_x->numel() == B * F * D, "out_x must be bf16 [B, F*D]");
      x = *out_x;
    } else {
      x = torch::empty({B, F * D}, table.options());
    }
  }
  if (want_fm) fm = torch::empty({B}, table.options().dtype(torch::kFloat32));
  dtfs::EmbedArgs a;
  a.table = table.data_ptr();
  a.lin = lin ? lin->data_ptr<float>() : nullptr;
  a.arena = arena.data_ptr();
  a.ids64 = true;
  a.B = int(B);
  a.F = int(F);
  a.D = int(D);
  a.V = V;
  a.modulo = modulo;
  a.bias = float(bias);
  a.out_x = want_x ? x.data_ptr() : nullptr;
  a.x_ld = F * D;
  a.out_fm = want_fm ? fm.data_ptr<float>() : nullptr;
  a.fm2 = fm2 ? 1 : 0;
  torch::Tensor q, qs;
  embed_fp8_out(a, table, B, F * D, k_pad, q, qs);
  TORCH_CHECK(!cross_w || want_fm, "cross: want_fm");
  embed_cross_in(a, table, F, D, cross_w, cross_c);
  check_hip(dtfs::launch_embed(a, cur_stream(table)), "embed_arena");
  return {x, fm, q, qs};
}

// ---------------------------------------------------------------- K1 fused into K4
// DeepFM / WDL first MLP layer straight from the table: the resolve kernel
// (ids / weights -> field-major rows / weights + first-order term) then the
// gather-GEMM (csrc/kernels/gemm.hip gemm_gather_kernel). Rows come from a
// device request arena (arena, B, F) or from ids [B, F] (+ wts). Returns
//   h     bf16 [B, N] = act(x . W^T + b), x = w * T[row] never materialised
//   parts fp32 [1 + (fm2 or cross), Mp]: row 0 = bias + first-order FM term,
//         row 1 the second-order FM term or (cross_w / cross_c: DCN v1's folded
//         cross weights) the cross logit; the head sums the rows.
// Request rows of a gather-GEMM: a device request arena, or ids (+ weights).
void embed_gemm_inputs(const torch::Tensor& table, const c10::optional<torch::Tensor>& arena,
                       const c10::optional<torch::Tensor>& ids, const c10::optional<torch::Tensor>& wts, int64_t B,
                       int64_t F, dtfs::EmbedArgs& a) {
  if (arena) {
    check_dev(*arena, "arena");
    check_same_dev(table, *arena, "arena");
    TORCH_CHECK(arena->scalar_type() == torch::kUInt8 && arena->is_contiguous() &&
                    arena->numel() > dtfs::kArenaPayloadOff,
                "arena must be a contiguous uint8 device buffer");
    TORCH_CHECK(!ids && !wts, "arena rows carry their own ids / weights");
    a.arena = arena->data_ptr();
  } else {
    TORCH_CHECK(ids.has_value(), "gather-GEMM needs an arena or ids");
    check_gpu(*ids, "ids");  // row views (e.g. the fan-out's narrow exchange rows) pass: strides checked below
    check_same_dev(table, *ids, "ids");
    TORCH_CHECK((ids->scalar_type() == torch::kInt64 || ids->scalar_type() == torch::kInt32) && ids->dim() == 2 &&
                    ids->size(0) == B && ids->size(1) == F && ids->stride(1) == 1 && ids->stride(0) >= F,
                "ids must be int32/int64 [B, F] with contiguous rows");
    a.ids = ids->data_ptr();
    a.ids64 = ids->scalar_type() == torch::kInt64;
    a.ids_ld = ids->stride(0);
    if (wts) {
      check_gpu(*wts, "wts");
      TORCH_CHECK(wts->scalar_type() == torch::kFloat32 && wts->dim() == 2 && wts->size(0) == B && wts->size(1) == F &&
                      wts->stride(1) == 1 && wts->stride(0) >= F,
                  "wts must be fp32 [B, F] with contiguous rows");
      a.wts = wts->data_ptr();
      a.wts_ld = wts->stride(0);
    }
  }
}

// K1 resolve into fresh field-major buffers (B rounded up to 256 rows).
std::vector<torch::Tensor> embed_gemm_resolve_into(const torch::Tensor& table, const c10::optional<torch::Tensor>& lin,
                                                   dtfs::EmbedArgs a, int64_t B, int64_t F, int64_t modulo,
                                                   double bias, int64_t n_parts) {
  const int64_t Mp = (B + 255) / 256 * 256;
  auto parts = torch::empty({n_parts, Mp}, table.options().dtype(torch::kFloat32));
  auto rows_t = torch::empty({F, Mp}, table.options().dtype(torch::kInt32));
  auto wts_t = torch::empty({F, Mp}, table.options().dtype(torch::kFloat32));
  if (B == 0) return {rows_t, wts_t, parts};
  a.table = table.data_ptr();
  a.lin = lin ? lin->data_ptr<float>() : nullptr;
  a.B = int(B);
  a.F = int(F);
  a.D = 64;
  a.V = table.size(0);
  a.modulo = modulo;
  a.bias = float(bias);
  check_hip(dtfs::launch_embed_resolve(a, rows_t.data_ptr<int32_t>(), wts_t.data_ptr<float>(), parts.data_ptr<float>(),
                                       Mp, cur_stream(table)),
            "embed_resolve");
  return {rows_t, wts_t, parts};
}

std::vector<torch::Tensor> embed_gemm(torch::Tensor table, c10::optional<torch::Tensor> lin,
                                      c10::optional<torch::Tensor> arena, c10::optional<torch::Tensor> ids,
                                      c10::optional<torch::Tensor> wts, int64_t B, int64_t F, int64_t modulo,
                                      double bias, torch::Tensor W, torch::Tensor b, int64_t act, bool fm2,
                                      c10::optional<torch::Tensor> cross_w, c10::optional<torch::Tensor> cross_c,
                                      c10::optional<std::vector<torch::Tensor>> resolved,
                                      c10::optional<torch::Tensor> Wp) {
  check_dev(table, "table");
  check_dev(W, "W");
  check_dev(b, "b");
  check_same_dev(table, W, "W");
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2 && table.size(1) == 64 &&
                  table.is_contiguous(),
              "gather-GEMM: table must be contiguous bf16 [V, 64]");
  const int64_t V = table.size(0);
  TORCH_CHECK(F >= 1 && F <= 64, "gather-GEMM handles 1..64 fields");
  TORCH_CHECK(modulo > 0 && modulo <= V, "modulo must be in (0, table rows]");
  TORCH_CHECK(W.scalar_type() == torch::kBFloat16 && W.dim() == 2 && W.size(1) == F * 64 && W.is_contiguous(),
              "W must be contiguous bf16 [N, 64 F]");
  const int64_t N = W.size(0);
  TORCH_CHECK(N % 256 == 0 && (!fm2 || N >= 1024), "gather-GEMM needs N % 256 == 0 (and N >= 1024 with FM)");
  TORCH_CHECK(b.scalar_type() == torch::kFloat32 && b.numel() == N, "b must be fp32 [N]");
  TORCH_CHECK(act == 0 || act == 1, "act must be 0 (none) or 1 (relu)");
  if (lin) {
    check_dev(*lin, "lin");
    TORCH_CHECK(lin->scalar_type() == torch::kFloat32 && lin->numel() == V, "lin must be fp32 [V]");
  }
  dtfs::EmbedArgs a;
  embed_gemm_inputs(table, arena, ids, wts, B, F, a);
  const bool cross = cross_w.has_value();
  if (cross) {
    check_dev(*cross_w, "cross_w");
    TORCH_CHECK(cross_c.has_value(), "cross_w and cross_c go together");
    check_dev(*cross_c, "cross_c");
    TORCH_CHECK(!fm2, "a model has either the FM term or the cross network");
    TORCH_CHECK(cross_w->scalar_type() == torch::kFloat32 && cross_w->dim() == 2 && cross_w->size(1) == F * 64 &&
                    cross_w->size(0) >= 1 && cross_w->size(0) <= 4 && cross_w->is_contiguous(),
                "cross_w must be contiguous fp32 [L + 1 <= 4, 64 F]");
    TORCH_CHECK(cross_c->scalar_type() == torch::kFloat32 && cross_c->numel() == cross_w->size(0),
                "cross_c must be fp32 [L + 1]");
    TORCH_CHECK(N >= 1024, "the cross network rides on N >= 1024 (4 column tiles)");
  }
  c10::DeviceGuard g(table.device());
  const int64_t Mp = (B + 255) / 256 * 256;
  auto h = torch::empty({B, N}, table.options());
  std::vector<torch::Tensor> r;
  if (resolved) {
    // the resolve pass ran earlier (embed_gemm_resolve, e.g. on another lane)
    r = *resolved;
    TORCH_CHECK(r.size() == 3, "resolved = (rows_t, wts_t, parts)");
    TORCH_CHECK(r[0].scalar_type() == torch::kInt32 && r[0].dim() == 2 && r[0].size(0) == F && r[0].size(1) == Mp &&
                    r[0].is_contiguous() && r[1].scalar_type() == torch::kFloat32 && r[1].sizes() == r[0].sizes() &&
                    r[1].is_contiguous() && r[2].scalar_type() == torch::kFloat32 && r[2].dim() == 2 &&
                    r[2].size(0) == ((fm2 || cross) ? 2 : 1) && r[2].size(1) == Mp && r[2].is_contiguous(),
                "resolved tensors do not match this gather-GEMM's shape");
    for (const auto& t : r) check_same_dev(table, t, "resolved");
  } else {
    r = embed_gemm_resolve_into(table, lin, a, B, F, modulo, bias, (fm2 || cross) ? 2 : 1);
  }
  const torch::Tensor &rows_t = r[0], &wts_t = r[1], &parts = r[2];
  if (B == 0) return {h, parts};
  auto st = cur_stream(table);
  if (Wp && dtfs::gemm_gather1w_ok(Mp, int(N), int(F), cross, V)) {
    // one wave per SIMD, B from registers (csrc/kernels/gather_gemm.hip)
    check_dev(*Wp, "Wp");
    check_same_dev(table, *Wp, "Wp");
    TORCH_CHECK(Wp->scalar_type() == torch::kBFloat16 && Wp->numel() == W.numel() && Wp->is_contiguous(),
                "Wp must be W packed in MFMA fragment order (ops.pack_bfrag)");
    check_hip(dtfs::launch_gemm_gather1w(table.data_ptr(), V, rows_t.data_ptr<int32_t>(), wts_t.data_ptr<float>(), Mp,
                                         int(F), Wp->data_ptr(), b.data_ptr<float>(), h.data_ptr(), N,
                                         fm2 ? parts.data_ptr<float>() : nullptr, int(B), int(N), int(act), st),
              "gemm_gather1w");
    return {h, parts};
  }
  check_hip(dtfs::launch_gemm_gather(table.data_ptr(), V, rows_t.data_ptr<int32_t>(), wts_t.data_ptr<float>(), Mp,
                                     int(F), W.data_ptr(), b.data_ptr<float>(), h.data_ptr(), N,
                                     (fm2 || cross) ? parts.data_ptr<float>() : nullptr, int(B), int(N), int(act), st,
                                     cross ? cross_w->data_ptr<float>() : nullptr,
                                     cross ? cross_c->data_ptr<float>() : nullptr, cross ? int(cross_w->size(0)) : 0),
            "gemm_gather");
  return {h, parts};
}

// The gather-GEMM's front half alone (K1 resolve): field-major table rows /
// weights + the first-order partial, for a gather-GEMM launched later (or on
// another stream: the step program's aux lane resolves step k+1 while the
// compute lane finishes step k).
std::vector<torch::Tensor> embed_gemm_resolve(torch::Tensor table, c10::optional<torch::Tensor> lin,
                                              c10::optional<torch::Tensor> arena, c10::optional<torch::Tensor> ids,
                                              c10::optional<torch::Tensor> wts, int64_t B, int64_t F, int64_t modulo,
                                              double bias, int64_t n_parts) {
  check_dev(table, "table");
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2 && table.size(1) == 64 &&
                  table.is_contiguous(),
              "gather-GEMM: table must be contiguous bf16 [V, 64]");
  TORCH_CHECK(F >= 1 && F <= 64, "gather-GEMM handles 1..64 fields");
  TORCH_CHECK(modulo > 0 && modulo <= table.size(0), "modulo must be in (0, table rows]");
  TORCH_CHECK(n_parts == 1 || n_parts == 2, "n_parts must be 1 or 2");
  if (lin) {
    check_dev(*lin, "lin");
    TORCH_CHECK(lin->scalar_type() == torch::kFloat32 && lin->numel() == table.size(0), "lin must be fp32 [V]");
  }
  dtfs::EmbedArgs a;
  embed_gemm_inputs(table, arena, ids, wts, B, F, a);
  c10::DeviceGuard g(table.device());
  return embed_gemm_resolve_into(table, lin, a, B, F, modulo, bias, n_parts);
}

// ---------------------------------------------------------------- K1b
torch::Tensor embedding_bag(torch::Tensor table, torch::Tensor idx, torch::Tensor offsets,
                            c10::optional<torch::Tensor> psw, int64_t modulo, bool mean, bool out_bf16,
                            c10::optional<torch::Tensor> out_opt) {
  check_dev(table, "table");
  check_dev(idx, "indices");
  check_dev(offsets, "offsets");
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2, "table must be bf16 [R, D]");
  TORCH_CHECK(idx.dim() == 1 && (idx.scalar_type() == torch::kInt64 || idx.scalar_type() == torch::kInt32),
              "indices must be int32/int64 [nnz]");
  TORCH_CHECK(offsets.dim() == 1 && offsets.scalar_type() == torch::kInt64 && offsets.numel() >= 1,
              "offsets must be int64 [nbags+1]");
  const int64_t D = table.size(1), R = table.size(0), nbags = offsets.numel() - 1;
  TORCH_CHECK(D == 8 || D == 16 || D == 32 || D == 64 || D == 128, "embedding dim must be 8/16/32/64/128");
  TORCH_CHECK(modulo > 0 && modulo <= R, "modulo must be in (0, rows]");
  // offsets are clamped into [0, nnz] inside the kernel (no host sync here)
  if (psw) {
    check_dev(*psw, "per_sample_weights");
    TORCH_CHECK(psw->scalar_type() == torch::kFloat32 && psw->numel() == idx.numel(), "per_sample_weights: fp32 [nnz]");
  }
  c10::DeviceGuard g(table.device());
  torch::Tensor out;
  if (out_opt) {  // a static buffer (captured steps: the exchange's send buffer)
    check_dev(*out_opt, "out");
    TORCH_CHECK(out_opt->scalar_type() == (out_bf16 ? torch::kBFloat16 : torch::kFloat32) && out_opt->is_contiguous() &&
                    out_opt->numel() == nbags * D,
                "out must be contiguous [nbags, D] of the output dtype");
    out = *out_opt;
  } else {
    out = torch::empty({nbags, D}, table.options().dtype(out_bf16 ? torch::kBFloat16 : torch::kFloat32));
  }
  check_hip(dtfs::launch_embedding_bag(table.data_ptr(), idx.data_ptr(), idx.scalar_type() == torch::kInt64,
                                       offsets.data_ptr<int64_t>(), psw ? psw->data_ptr<float>() : nullptr, int(nbags),
                                       idx.numel(), int(D), modulo, mean, out_bf16 ? nullptr : out.data_ptr<float>(),
                                       out_bf16 ? out.data_ptr() : nullptr, D, cur_stream(table)),
            "embedding_bag");
  return out;
}

// ---------------------------------------------------------------- K4 / K3b
torch::Tensor gemm(torch::Tensor A, torch::Tensor W, c10::optional<torch::Tensor> bias, int64_t epi,
                   c10::optional<torch::Tensor> x0, c10::optional<torch::Tensor> xl, bool out_f32,
                   c10::optional<torch::Tensor> sa, c10::optional<torch::Tensor> sw, c10::optional<torch::Tensor> out,
                   int64_t variant, c10::optional<torch::Tensor> sa_blk, c10::optional<torch::Tensor> q_out,
                   c10::optional<torch::Tensor> sq_out) {
  check_dev(A, "A");
  check_dev(W, "W");
  check_same_dev(A, W, "W");
  TORCH_CHECK(A.dim() == 2 && W.dim() == 2, "A [M,K], W [N,K]");
  const bool fp8 = A.scalar_type() == torch::kFloat8_e4m3fn || A.scalar_type() == torch::kUInt8;
  if (fp8) {
    TORCH_CHECK(W.scalar_type() == A.scalar_type(), "fp8 GEMM needs fp8 (e4m3fn) A and W");
    TORCH_CHECK((sa.has_value() || sa_blk.has_value()) && sw.has_value(),
                "fp8 GEMM needs row scales sa [M] (or MX block scales sa_blk) and channel scales sw [N]");
  } else {
    TORCH_CHECK(!sa_blk && !q_out, "MX block scales are an fp8-path feature");
    TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && W.scalar_type() == torch::kBFloat16, "bf16 GEMM needs bf16 A, W");
  }
  const int64_t M = A.size(0), K = A.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "K mismatch: A ", A.sizes(), " W ", W.sizes());
  TORCH_CHECK(fp8 ? K % 16 == 0 : K % 8 == 0, "K must be a multiple of 16 bytes");
  TORCH_CHECK(M < (int64_t(1) << 31) && N < (int64_t(1) << 31), "dims too large");
  if (bias) {
    check_dev(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == N, "bias must be fp32 [N]");
  }
  if (sa) {
    check_dev(*sa, "sa");
    TORCH_CHECK(sa->scalar_type() == torch::kFloat32 && sa->numel() == M, "sa must be fp32 [M]");
  }
  if (sw) {
    check_dev(*sw, "sw");
    TORCH_CHECK(sw->scalar_type() == torch::kFloat32 && sw->numel() == N, "sw must be fp32 [N]");
  }
  TORCH_CHECK((epi & 15) <= 3 && epi >= 0 && epi < 32, "epi must be 0..3 (+16: M-fastest tile order)");
  if ((epi & 15) == 3) {
    TORCH_CHECK(x0.has_value() && xl.has_value(), "cross epilogue needs x0 and xl");
    for (auto* t : {&x0, &xl}) {
      check_dev(**t, "x0/xl");
      TORCH_CHECK((*t)->scalar_type() == torch::kBFloat16 && (*t)->size(0) == M && (*t)->size(1) == N,
                  "x0/xl must be bf16 [M, N]");
    }
  }
  dtfs::MxIO mx;
  if (sa_blk) {
    check_dev(*sa_blk, "sa_blk");
    TORCH_CHECK(sa_blk->scalar_type() == torch::kUInt8 && sa_blk->dim() == 2 && sa_blk->size(0) == M &&
                    sa_blk->size(1) >= K / 32 && sa_blk->stride(1) == 1 && sa_blk->stride(0) % 4 == 0 &&
                    reinterpret_cast<uintptr_t>(sa_blk->data_ptr()) % 4 == 0,
                "sa_blk must be uint8 [M, >= K/32] (E8M0 per 32 K elements)");
    TORCH_CHECK(K % 128 == 0 && K <= 3072, "MX block scales need K % 128 == 0 and K <= 3072");
    mx.sab = sa_blk->data_ptr<uint8_t>();
    mx.ldsab = sa_blk->stride(0);
  }
  if (q_out) {
    TORCH_CHECK(sq_out.has_value() && (epi & 15) == 3, "q_out needs sq_out and the cross epilogue");
    check_dev(*q_out, "q_out");
    check_dev(*sq_out, "sq_out");
    TORCH_CHECK((q_out->scalar_type() == torch::kFloat8_e4m3fn || q_out->scalar_type() == torch::kUInt8) &&
                    q_out->dim() == 2 && q_out->size(0) == M && q_out->size(1) >= N && q_out->size(1) % 32 == 0 &&
                    q_out->stride(1) == 1 && q_out->stride(0) % 4 == 0,
                "q_out must be e4m3 [M, >= N, multiple of 32]");
    TORCH_CHECK(sq_out->scalar_type() == torch::kUInt8 && sq_out->dim() == 2 && sq_out->size(0) == M &&
                    sq_out->size(1) >= q_out->size(1) / 32 && sq_out->stride(1) == 1,
                "sq_out must be uint8 [M, >= q columns / 32]");
    TORCH_CHECK(N % 32 == 0, "MX output needs N % 32 == 0");
    mx.q = static_cast<uint8_t*>(q_out->data_ptr());
    mx.ldq = q_out->stride(0);
    mx.sq = sq_out->data_ptr<uint8_t>();
    mx.ldsq = sq_out->stride(0);
    mx.nq = int(q_out->size(1));
  }
  c10::DeviceGuard g(A.device());
  torch::Tensor C;
  if (out) {
    check_dev(*out, "out");
    TORCH_CHECK(out->size(0) == M && out->size(1) == N, "out must be [M, N]");
    TORCH_CHECK(out->scalar_type() == (out_f32 ? torch::kFloat32 : torch::kBFloat16), "out dtype mismatch");
    C = *out;
  } else {
    C = torch::empty({M, N}, A.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  }
  check_hip(dtfs::launch_gemm(A.data_ptr(), K, W.data_ptr(), K, bias ? bias->data_ptr<float>() : nullptr,
                              sa ? sa->data_ptr<float>() : nullptr, sw ? sw->data_ptr<float>() : nullptr, C.data_ptr(),
                              N, out_f32, opt_ptr(x0), opt_ptr(xl), N, int(M), int(N), int(K), int(epi), fp8,
                              cur_stream(A), int(variant), (sa_blk || q_out) ? &mx : nullptr),
            "gemm");
  return C;
}

// ---------------------------------------------------------------- K3
std::vector<torch::Tensor> cross_v1(torch::Tensor x0, torch::Tensor w, torch::Tensor b, bool want_x,
                                    c10::optional<torch::Tensor> head_w) {
  check_dev(x0, "x0");
  check_dev(w, "w");
  check_dev(b, "b");
  TORCH_CHECK(x0.scalar_type() == torch::kBFloat16 && x0.dim() == 2, "x0 must be bf16 [B, d]");
  const int64_t B = x0.size(0), d = x0.size(1);
  TORCH_CHECK(d % 8 == 0 && d <= 64 * 8 * 8, "d must be a multiple of 8 and <= 4096");
  TORCH_CHECK(w.scalar_type() == torch::kFloat32 && w.dim() == 2 && w.size(1) == d, "w must be fp32 [L, d]");
  TORCH_CHECK(b.scalar_type() == torch::kFloat32 && b.sizes() == w.sizes(), "b must be fp32 [L, d]");
  if (head_w) {
    check_dev(*head_w, "head_w");
    TORCH_CHECK(head_w->scalar_type() == torch::kFloat32 && head_w->numel() == d, "head_w must be fp32 [d]");
  }
  c10::DeviceGuard g(x0.device());
  torch::Tensor x, dot;
  if (want_x) x = torch::empty_like(x0);
  if (head_w) dot = torch::empty({B}, x0.options().dtype(torch::kFloat32));
  check_hip(dtfs::launch_cross_v1(x0.data_ptr(), d, int(B), int(d), int(w.size(0)), w.data_ptr<float>(),
                                  b.data_ptr<float>(), want_x ? x.data_ptr() : nullptr, d,
                                  head_w ? head_w->data_ptr<float>() : nullptr,
                                  head_w ? dot.data_ptr<float>() : nullptr, cur_stream(x0)),
            "cross_v1");
  return {x, dot};
}

// ---------------------------------------------------------------- K5
torch::Tensor dot_interaction(torch::Tensor dense, torch::Tensor emb, int64_t out_cols,
                              c10::optional<torch::Tensor> emb_off, c10::optional<torch::Tensor> emb_stride) {
  check_dev(dense, "dense");
  check_dev(emb, "emb");
  TORCH_CHECK(dense.scalar_type() == torch::kBFloat16 && emb.scalar_type() == torch::kBFloat16, "bf16 inputs");
  TORCH_CHECK(dense.dim() == 2 && dense.size(1) == 64, "dense must be [B, 64]");
  const int64_t B = dense.size(0);
  int64_t T;
  if (emb_off.has_value() || emb_stride.has_value()) {
    // table map: emb is a flat [N, 64] buffer; table t of row b is row off[t] + b * stride[t]
    TORCH_CHECK(emb_off.has_value() && emb_stride.has_value(), "emb_off and emb_stride go together");
    TORCH_CHECK(emb.dim() == 2 && emb.size(1) == 64, "mapped emb must be a flat [N, 64] buffer");
    for (auto* o : {&emb_off, &emb_stride}) {
      check_dev(**o, "table map");
      TORCH_CHECK((*o)->scalar_type() == torch::kInt64 && (*o)->dim() == 1, "table map entries are int64 [T]");
    }
    T = emb_off->numel();
    TORCH_CHECK(emb_stride->numel() == T, "emb_off and emb_stride must have T entries");
    // the kernel clamps every mapped row into [0, N): no host sync here, so
    // this call is capturable into a step graph
  } else {
    TORCH_CHECK(emb.dim() == 3 && emb.size(0) == B && emb.size(2) == 64, "emb must be [B, T, 64]");
    T = emb.size(1);
  }
  TORCH_CHECK(T + 1 <= 32, "dot interaction kernel handles T + 1 <= 32 vectors");
  const int64_t used = 64 + (T + 1) * T / 2;
  if (out_cols <= 0) out_cols = (used + 7) / 8 * 8;
  TORCH_CHECK(out_cols >= used, "out_cols too small");
  c10::DeviceGuard g(dense.device());
  auto out = torch::empty({B, out_cols}, dense.options());
  check_hip(dtfs::launch_dot_interaction(dense.data_ptr(), 64, emb.data_ptr(), int(T), int(B), out.data_ptr(),
                                         out_cols, int(out_cols), cur_stream(dense),
                                         emb_off ? emb_off->data_ptr<int64_t>() : nullptr,
                                         emb_stride ? emb_stride->data_ptr<int64_t>() : nullptr, emb.size(0)),
            "dot_interaction");
  return out;
}

// K1 + K5: dot interaction straight from the (local, one-hot) tables
torch::Tensor dot_interaction_gather(torch::Tensor dense, torch::Tensor table, torch::Tensor ids,
                                     torch::Tensor modulo_f, torch::Tensor offset_f, int64_t out_cols) {
  check_dev(dense, "dense");
  check_same_dev(dense, table, "table");
  check_same_dev(dense, ids, "ids");
  TORCH_CHECK(dense.scalar_type() == torch::kBFloat16 && table.scalar_type() == torch::kBFloat16, "bf16 inputs");
  TORCH_CHECK(dense.dim() == 2 && dense.size(1) == 64 && dense.stride(1) == 1 && dense.stride(0) % 8 == 0,
              "dense must be [B, 64] with unit inner stride");
  TORCH_CHECK(table.dim() == 2 && table.size(1) == 64 && table.is_contiguous(), "table must be contiguous [V, 64]");
  TORCH_CHECK((ids.scalar_type() == torch::kInt64 || ids.scalar_type() == torch::kInt32) && ids.dim() == 2 &&
                  ids.stride(1) == 1 && ids.size(0) == dense.size(0),
              "ids must be int32/int64 [B, T] rows with unit inner stride");
  const int64_t B = dense.size(0), T = ids.size(1);
  for (auto* t : {&modulo_f, &offset_f}) {
    check_same_dev(dense, *t, "table map");
    TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->numel() == T && t->is_contiguous(), "modulo_f / offset_f: int64 [T]");
  }
  TORCH_CHECK(T + 1 <= 32, "dot interaction kernel handles T + 1 <= 32 vectors");
  const int64_t used = 64 + (T + 1) * T / 2;
  if (out_cols <= 0) out_cols = (used + 7) / 8 * 8;
  TORCH_CHECK(out_cols >= used && out_cols % 8 == 0 && out_cols <= 1024, "out_cols: >= used, a multiple of 8, <= 1024");
  c10::DeviceGuard g(dense.device());
  auto out = torch::empty({B, out_cols}, dense.options());
  check_hip(dtfs::launch_dot_interaction_gather(dense.data_ptr(), dense.stride(0), table.data_ptr(), table.size(0),
                                                ids.data_ptr(), ids.scalar_type() == torch::kInt64, ids.stride(0),
                                                modulo_f.data_ptr<int64_t>(), offset_f.data_ptr<int64_t>(), int(T),
                                                int(B), out.data_ptr(), out_cols, int(out_cols), cur_stream(dense)),
            "dot_interaction_gather");
  return out;
}

// DLRM bottom MLP (512-256-64, relu) from the fp32 dense feature columns, one
// kernel. arena (uint8 device request arena, M = its first M rows) replaces wts.
static torch::Tensor bottom_mlp3_impl(const torch::Tensor* wts, const torch::Tensor* arena, int64_t M, int64_t nd,
                                      torch::Tensor W1, torch::Tensor b1, torch::Tensor W2, torch::Tensor b2,
                                      torch::Tensor W3, torch::Tensor b3) {
  const torch::Tensor& ref = wts ? *wts : *arena;
  TORCH_CHECK(ref.is_cuda(), "bottom MLP input must be a GPU tensor");
  if (wts) {
    TORCH_CHECK(wts->scalar_type() == torch::kFloat32 && wts->dim() == 2 && wts->stride(1) == 1 && wts->size(1) >= nd,
                "wts must be fp32 [M, >= nd] rows with unit inner stride");
  } else {
    TORCH_CHECK(arena->scalar_type() == torch::kUInt8 && arena->is_contiguous(), "arena must be a contiguous uint8 buffer");
  }
  const torch::Tensor& wts_ = ref;
  const torch::Tensor* Ws[3] = {&W1, &W2, &W3};
  const torch::Tensor* bs[3] = {&b1, &b2, &b3};
  int64_t k = 64;
  for (int i = 0; i < 3; ++i) {
    check_same_dev(wts_, *Ws[i], "weight");
    check_same_dev(wts_, *bs[i], "bias");
    TORCH_CHECK(Ws[i]->scalar_type() == torch::kBFloat16 && Ws[i]->dim() == 2 && Ws[i]->is_contiguous() &&
                    Ws[i]->size(1) == k,
                "bottom MLP weight ", i, " must be contiguous bf16 [N, ", k, "]");
    TORCH_CHECK(bs[i]->scalar_type() == torch::kFloat32 && bs[i]->numel() == Ws[i]->size(0) && bs[i]->is_contiguous(),
                "bottom MLP bias must be fp32 [N]");
    k = Ws[i]->size(0);
  }
  const int64_t N3 = W3.size(0);
  c10::DeviceGuard g(wts_.device());
  auto out = torch::empty({M, N3}, W1.options());
  check_hip(dtfs::launch_bottom_mlp3(wts ? wts->data_ptr<float>() : nullptr, wts ? wts->stride(0) : 0, int(nd),
                                     int(M), W1.data_ptr(), b1.data_ptr<float>(), int(W1.size(0)), W2.data_ptr(),
                                     b2.data_ptr<float>(), int(W2.size(0)), W3.data_ptr(), b3.data_ptr<float>(),
                                     int(N3), out.data_ptr(), N3, cur_stream(wts_),
                                     arena ? arena->data_ptr() : nullptr),
            "bottom_mlp3");
  return out;
}

torch::Tensor bottom_mlp3(torch::Tensor wts, int64_t nd, torch::Tensor W1, torch::Tensor b1, torch::Tensor W2,
                          torch::Tensor b2, torch::Tensor W3, torch::Tensor b3) {
  return bottom_mlp3_impl(&wts, nullptr, wts.size(0), nd, W1, b1, W2, b2, W3, b3);
}

torch::Tensor bottom_mlp3_arena(torch::Tensor arena, int64_t B, int64_t nd, torch::Tensor W1, torch::Tensor b1,
                                torch::Tensor W2, torch::Tensor b2, torch::Tensor W3, torch::Tensor b3) {
  return bottom_mlp3_impl(nullptr, &arena, B, nd, W1, b1, W2, b2, W3, b3);
}

// the dot interaction with its ids read from a device request arena (features
// id_col0 .. id_col0 + T - 1 of each row)
torch::Tensor dot_interaction_gather_arena(torch::Tensor dense, torch::Tensor table, torch::Tensor arena,
                                           int64_t id_col0, torch::Tensor modulo_f, torch::Tensor offset_f,
                                           int64_t out_cols) {
  check_dev(dense, "dense");
  check_same_dev(dense, table, "table");
  check_same_dev(dense, arena, "arena");
  TORCH_CHECK(arena.scalar_type() == torch::kUInt8 && arena.is_contiguous(), "arena must be a contiguous uint8 buffer");
  TORCH_CHECK(dense.scalar_type() == torch::kBFloat16 && table.scalar_type() == torch::kBFloat16, "bf16 inputs");
  TORCH_CHECK(dense.dim() == 2 && dense.size(1) == 64, "dense must be [B, 64]");
  TORCH_CHECK(table.dim() == 2 && table.size(1) == 64 && table.is_contiguous(), "table must be contiguous [V, 64]");
  const int64_t B = dense.size(0), T = modulo_f.numel();
  for (auto* t : {&modulo_f, &offset_f}) {
    check_same_dev(dense, *t, "table map");
    TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->numel() == T && t->is_contiguous(), "modulo_f / offset_f: int64 [T]");
  }
  TORCH_CHECK(T >= 1 && T + 1 <= 32 && id_col0 >= 0, "1 <= T <= 31 tables, id_col0 >= 0");
  const int64_t used = 64 + (T + 1) * T / 2;
  if (out_cols <= 0) out_cols = (used + 7) / 8 * 8;
  TORCH_CHECK(out_cols >= used && out_cols % 8 == 0 && out_cols <= 1024, "out_cols: >= used, a multiple of 8, <= 1024");
  c10::DeviceGuard g(dense.device());
  auto out = torch::empty({B, out_cols}, dense.options());
  check_hip(dtfs::launch_dot_interaction_gather(dense.data_ptr(), 64, table.data_ptr(), table.size(0), nullptr, true, 0,
                                                modulo_f.data_ptr<int64_t>(), offset_f.data_ptr<int64_t>(), int(T),
                                                int(B), out.data_ptr(), out_cols, int(out_cols), cur_stream(dense),
                                                arena.data_ptr(), int(id_col0)),
            "dot_interaction_gather_arena");
  return out;
}

// ---------------------------------------------------------------- K1b routing
torch::Tensor shard_route(c10::optional<torch::Tensor> ids, c10::optional<torch::Tensor> arena, int64_t B, int64_t F,
                          int64_t W, int64_t tm, torch::Tensor col, torch::Tensor mod, torch::Tensor off,
                          c10::optional<torch::Tensor> out_opt, int64_t hot, c10::optional<torch::Tensor> wts,
                          c10::optional<torch::Tensor> out_w) {
  TORCH_CHECK(ids.has_value() != arena.has_value(), "shard_route: ids or a device arena");
  TORCH_CHECK(W >= 1 && tm >= 1 && hot >= 1 && B >= 0 && F >= 1, "W, tm, hot, F >= 1");
  dtfs::RouteArgs a;
  torch::Tensor ref;
  if (ids) {
    TORCH_CHECK(ids->is_cuda() && ids->dim() == 2 && ids->stride(1) == 1 && ids->stride(0) >= ids->size(1),
                "ids must be a GPU [B, F] row view with contiguous rows");
    TORCH_CHECK(ids->scalar_type() == torch::kInt64 || ids->scalar_type() == torch::kInt32, "ids must be int32/int64");
    TORCH_CHECK(ids->size(0) == B && ids->size(1) == F, "ids must be [B, F]");
    a.ids = ids->data_ptr();
    a.ids64 = ids->scalar_type() == torch::kInt64;
    a.ld = ids->stride(0);
    ref = *ids;
    if (wts) {
      check_dev(*wts, "wts");
      TORCH_CHECK(wts->scalar_type() == torch::kFloat32 && wts->dim() == 2 && wts->size(0) == B &&
                      wts->size(1) == F && wts->stride(1) == 1,
                  "wts must be fp32 [B, F] with contiguous rows");
      a.wts = wts->data_ptr<float>();
      a.wts_ld = wts->stride(0);
    }
  } else {
    check_dev(*arena, "arena");
    TORCH_CHECK(arena->scalar_type() == torch::kUInt8 && arena->is_contiguous() && arena->numel() > dtfs::kArenaPayloadOff,
                "arena must be a contiguous uint8 device buffer");
    TORCH_CHECK(!wts, "arena rows carry their own weights");
    a.arena = arena->data_ptr<uint8_t>();
    ref = *arena;
  }
  check_dev(col, "col");
  check_dev(mod, "mod");
  check_dev(off, "off");
  TORCH_CHECK(col.scalar_type() == torch::kInt32 && col.numel() == W * tm, "col must be int32 [W * tm]");
  TORCH_CHECK(mod.scalar_type() == torch::kInt64 && mod.numel() == W * tm, "mod must be int64 [W * tm]");
  TORCH_CHECK(off.scalar_type() == torch::kInt64 && off.numel() == W * tm, "off must be int64 [W * tm]");
  check_same_dev(ref, col, "col");
  // route columns are clamped into [0, F) by the kernel (capturable: no sync)
  c10::DeviceGuard g(ref.device());
  torch::Tensor out;
  const int64_t n = W * B * tm * hot;
  if (out_opt) {
    check_dev(*out_opt, "out");
    TORCH_CHECK(out_opt->scalar_type() == torch::kInt32 && out_opt->numel() == n && out_opt->is_contiguous(),
                "out must be contiguous int32 [W, B, tm * hot]");
    check_same_dev(ref, *out_opt, "out");
    out = *out_opt;
  } else {
    out = torch::empty({W, B, tm * hot}, ref.options().dtype(torch::kInt32));
  }
  if (out_w) {
    check_dev(*out_w, "out_w");
    TORCH_CHECK(out_w->scalar_type() == torch::kFloat32 && out_w->numel() == n && out_w->is_contiguous(),
                "out_w must be contiguous fp32 [W, B, tm * hot]");
    a.out_w = out_w->data_ptr<float>();
  }
  a.B = int(B);
  a.F = int(F);
  a.W = int(W);
  a.tm = int(tm);
  a.hot = int(hot);
  a.col = col.data_ptr<int32_t>();
  a.mod = mod.data_ptr<int64_t>();
  a.off = off.data_ptr<int64_t>();
  a.out = out.data_ptr<int32_t>();
  check_hip(dtfs::launch_shard_route(a, cur_stream(ref)), "shard_route");
  return out;
}

// ---------------------------------------------------------------- peer lookup
// PeerTables (parallel/hot_cache.py): cbase int64 [W * max_chunks] (device
// addresses of every rank's store chunks), towner int32 [T], toff int64 [T],
// trows int64 [T], tremote int32 [T]; the replica cache: cache int64 [5],
// stats int64 [128], ring int64 [cap] (64 segments), ring_ctr int64 [64]
static dtfs::PeerLookupArgs peer_args(const torch::Tensor& ref, const torch::Tensor& cbase,
                                      const torch::Tensor& towner, const torch::Tensor& toff,
                                      const torch::Tensor& trows, const torch::Tensor& tremote, int64_t chunk_shift,
                                      const c10::optional<torch::Tensor>& cache,
                                      const c10::optional<torch::Tensor>& stats,
                                      const c10::optional<torch::Tensor>& ring,
                                      const c10::optional<torch::Tensor>& ring_ctr, int64_t sample_every) {
  const int64_t T = trows.numel();
  for (auto* t : {&cbase, &toff, &trows}) {
    check_same_dev(ref, *t, "peer table map");
    TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->is_contiguous(), "cbase / toff / trows: contiguous int64");
  }
  for (auto* t : {&towner, &tremote}) {
    check_same_dev(ref, *t, "peer table map");
    TORCH_CHECK(t->scalar_type() == torch::kInt32 && t->numel() == T && t->is_contiguous(), "towner / tremote: int32 [T]");
  }
  TORCH_CHECK(toff.numel() == T && cbase.numel() >= 1, "toff: int64 [T], cbase: int64 [W * max_chunks]");
  TORCH_CHECK(chunk_shift >= 1 && chunk_shift <= 40, "chunk_shift in [1, 40]");
  dtfs::PeerLookupArgs p;
  p.cbase = cbase.data_ptr<int64_t>();
  p.towner = towner.data_ptr<int32_t>();
  p.toff = toff.data_ptr<int64_t>();
  p.trows = trows.data_ptr<int64_t>();
  p.tremote = tremote.data_ptr<int32_t>();
  p.chunk_shift = int(chunk_shift);
  p.max_chunks = int(cbase.size(-1));
  TORCH_CHECK(cbase.dim() == 2, "cbase must be [W, max_chunks]");
  if (cache) {
    check_same_dev(ref, *cache, "cache");
    TORCH_CHECK(cache->scalar_type() == torch::kInt64 && cache->numel() == 5 && cache->is_contiguous(), "cache: int64 [5]");
    p.cache = cache->data_ptr<int64_t>();
  }
  if (stats) {
    check_same_dev(ref, *stats, "stats");
    TORCH_CHECK(stats->scalar_type() == torch::kInt64 && stats->numel() == 128 && stats->is_contiguous(),
                "stats: int64 [128]");
    p.stats = reinterpret_cast<unsigned long long*>(stats->data_ptr<int64_t>());
  }
  if (ring) {
    TORCH_CHECK(ring_ctr.has_value(), "ring needs ring_ctr");
    check_same_dev(ref, *ring, "ring");
    check_same_dev(ref, *ring_ctr, "ring_ctr");
    TORCH_CHECK(ring->scalar_type() == torch::kInt64 && ring->numel() >= 64 && ring->numel() % 64 == 0 &&
                    ring->is_contiguous(),
                "ring: int64 [cap], cap a multiple of 64");
    TORCH_CHECK(ring_ctr->scalar_type() == torch::kInt64 && ring_ctr->numel() == 64 && ring_ctr->is_contiguous(),
                "ring_ctr: int64 [64]");
    p.ring = ring->data_ptr<int64_t>();
    p.ring_ctr = reinterpret_cast<unsigned long long*>(ring_ctr->data_ptr<int64_t>());
    p.ring_cap = ring->numel();
    p.sample_every = int(std::max<int64_t>(sample_every, 0));
  }
  return p;
}

// K1 + K5 through the peer lookup: ids [B, >= id_col0 + T] int32/int64 rows,
// or a device request arena (B rows)
torch::Tensor dot_interaction_gather_peer(torch::Tensor dense, c10::optional<torch::Tensor> ids,
                                          c10::optional<torch::Tensor> arena, int64_t id_col0, torch::Tensor cbase,
                                          torch::Tensor towner, torch::Tensor toff, torch::Tensor trows,
                                          torch::Tensor tremote, int64_t chunk_shift,
                                          c10::optional<torch::Tensor> cache, c10::optional<torch::Tensor> stats,
                                          c10::optional<torch::Tensor> ring, c10::optional<torch::Tensor> ring_ctr,
                                          int64_t sample_every, int64_t out_cols) {
  check_dev(dense, "dense");
  TORCH_CHECK(ids.has_value() != arena.has_value(), "dot_interaction_gather_peer: ids or a device arena");
  TORCH_CHECK(dense.scalar_type() == torch::kBFloat16 && dense.dim() == 2 && dense.size(1) == 64 &&
                  dense.stride(1) == 1 && dense.stride(0) % 8 == 0,
              "dense must be bf16 [B, 64] with unit inner stride");
  const int64_t B = dense.size(0), T = trows.numel();
  TORCH_CHECK(T >= 1 && T + 1 <= 32 && id_col0 >= 0, "1 <= T <= 31 tables, id_col0 >= 0");
  const void* idp = nullptr;
  bool ids64 = true;
  int64_t ldi = 0;
  if (ids) {
    check_same_dev(dense, *ids, "ids");
    TORCH_CHECK((ids->scalar_type() == torch::kInt64 || ids->scalar_type() == torch::kInt32) && ids->dim() == 2 &&
                    ids->stride(1) == 1 && ids->size(0) == B && ids->size(1) >= id_col0 + T,
                "ids must be int32/int64 [B, >= id_col0 + T] rows with unit inner stride");
    ids64 = ids->scalar_type() == torch::kInt64;
    ldi = ids->stride(0);
    idp = static_cast<const uint8_t*>(ids->data_ptr()) + id_col0 * ids->element_size();
  } else {
    check_same_dev(dense, *arena, "arena");
    TORCH_CHECK(arena->scalar_type() == torch::kUInt8 && arena->is_contiguous(), "arena must be a contiguous uint8 buffer");
  }
  const auto p = peer_args(dense, cbase, towner, toff, trows, tremote, chunk_shift, cache, stats, ring, ring_ctr,
                           sample_every);
  const int64_t used = 64 + (T + 1) * T / 2;
  if (out_cols <= 0) out_cols = (used + 7) / 8 * 8;
  TORCH_CHECK(out_cols >= used && out_cols % 8 == 0 && out_cols <= 1024, "out_cols: >= used, a multiple of 8, <= 1024");
  c10::DeviceGuard g(dense.device());
  auto out = torch::empty({B, out_cols}, dense.options());
  check_hip(dtfs::launch_dot_interaction_gather(dense.data_ptr(), dense.stride(0), nullptr, 0, idp, ids64, ldi, nullptr,
                                                nullptr, int(T), int(B), out.data_ptr(), out_cols, int(out_cols),
                                                cur_stream(dense), arena ? arena->data_ptr() : nullptr,
                                                arena ? int(id_col0) : 0, &p),
            "dot_interaction_gather_peer");
  return out;
}

// K1b through the peer lookup: pooled bags -> out bf16 [B, T, 64]
void peer_bag(c10::optional<torch::Tensor> ids, c10::optional<torch::Tensor> wts, c10::optional<torch::Tensor> arena,
              int64_t B, int64_t col0, int64_t hot, torch::Tensor cbase, torch::Tensor towner, torch::Tensor toff,
              torch::Tensor trows, torch::Tensor tremote, int64_t chunk_shift, c10::optional<torch::Tensor> cache, c10::optional<torch::Tensor> stats, c10::optional<torch::Tensor> ring,
              c10::optional<torch::Tensor> ring_ctr, int64_t sample_every, torch::Tensor out) {
  check_dev(out, "out");
  TORCH_CHECK(ids.has_value() != arena.has_value(), "peer_bag: ids (+ wts) or a device arena");
  const int64_t T = trows.numel();
  TORCH_CHECK(T >= 1 && hot >= 1 && col0 >= 0 && B >= 0, "T, hot >= 1, col0 >= 0");
  TORCH_CHECK(out.scalar_type() == torch::kBFloat16 && out.is_contiguous() && out.numel() == B * T * 64,
              "out must be contiguous bf16 [B, T, 64]");
  const void* idp = nullptr;
  const float* wp = nullptr;
  bool ids64 = true;
  int64_t ldi = 0, ldw = 0;
  const int64_t need = col0 + T * hot;
  if (ids) {
    TORCH_CHECK(wts.has_value(), "peer_bag: ids need wts");
    check_same_dev(out, *ids, "ids");
    check_same_dev(out, *wts, "wts");
    TORCH_CHECK((ids->scalar_type() == torch::kInt64 || ids->scalar_type() == torch::kInt32) && ids->dim() == 2 &&
                    ids->stride(1) == 1 && ids->size(0) == B && ids->size(1) >= need,
                "ids must be int32/int64 [B, >= col0 + T * hot] rows with unit inner stride");
    TORCH_CHECK(wts->scalar_type() == torch::kFloat32 && wts->dim() == 2 && wts->stride(1) == 1 && wts->size(0) == B &&
                    wts->size(1) >= need,
                "wts must be fp32 [B, >= col0 + T * hot] rows with unit inner stride");
    ids64 = ids->scalar_type() == torch::kInt64;
    idp = ids->data_ptr();
    ldi = ids->stride(0);
    wp = wts->data_ptr<float>();
    ldw = wts->stride(0);
  } else {
    check_same_dev(out, *arena, "arena");
    TORCH_CHECK(arena->scalar_type() == torch::kUInt8 && arena->is_contiguous(), "arena must be a contiguous uint8 buffer");
  }
  const auto p = peer_args(out, cbase, towner, toff, trows, tremote, chunk_shift, cache, stats, ring, ring_ctr,
                           sample_every);
  c10::DeviceGuard g(out.device());
  check_hip(dtfs::launch_peer_bag(p, idp, ids64, ldi, wp, ldw, arena ? arena->data_ptr() : nullptr, int(col0), int(T),
                                  int(hot), int(B), out.data_ptr(), cur_stream(out)),
            "peer_bag");
}

// replica cache maintenance (parallel/hot_cache.py)
void peer_cache_fill(torch::Tensor keys, torch::Tensor slots, torch::Tensor cbase, torch::Tensor towner,
                     torch::Tensor toff, torch::Tensor trows, torch::Tensor tremote, int64_t chunk_shift,
                     torch::Tensor rows) {
  check_dev(rows, "rows");
  for (auto* t : {&keys, &slots}) check_same_dev(rows, *t, "cache fill input");
  TORCH_CHECK(keys.scalar_type() == torch::kInt64 && keys.is_contiguous() && slots.scalar_type() == torch::kInt32 &&
                  slots.is_contiguous() && slots.numel() == keys.numel(),
              "keys int64 [n], slots int32 [n]");
  TORCH_CHECK(rows.scalar_type() == torch::kBFloat16 && rows.dim() == 2 && rows.size(1) == 64 && rows.is_contiguous(),
              "rows must be contiguous bf16 [cap, 64]");
  const auto p = peer_args(rows, cbase, towner, toff, trows, tremote, chunk_shift, c10::nullopt, c10::nullopt,
                           c10::nullopt, c10::nullopt, 0);
  c10::DeviceGuard g(rows.device());
  check_hip(dtfs::launch_peer_cache_fill(p, int(trows.numel()), keys.data_ptr<int64_t>(), slots.data_ptr<int32_t>(),
                                         keys.numel(), rows.data_ptr(), rows.size(0), cur_stream(rows)),
            "peer_cache_fill");
}

void cache_index_build(torch::Tensor keys, torch::Tensor slots, torch::Tensor entries) {
  check_dev(entries, "entries");
  for (auto* t : {&keys, &slots}) check_same_dev(entries, *t, "cache index input");
  TORCH_CHECK(keys.scalar_type() == torch::kInt64 && keys.is_contiguous() && slots.scalar_type() == torch::kInt32 &&
                  slots.is_contiguous() && slots.numel() == keys.numel(),
              "keys int64 [n], slots int32 [n]");
  TORCH_CHECK(entries.scalar_type() == torch::kInt64 && entries.is_contiguous() && entries.numel() % 2 == 0,
              "entries: int64 [H, 2]");
  const int64_t H = entries.numel() / 2;
  TORCH_CHECK(H >= 2 && (H & (H - 1)) == 0 && 2 * keys.numel() <= H, "index size: a power of two >= 2 n");
  c10::DeviceGuard g(entries.device());
  check_hip(dtfs::launch_cache_index_build(keys.data_ptr<int64_t>(), slots.data_ptr<int32_t>(), keys.numel(),
                                           entries.data_ptr<int64_t>(), H - 1, cur_stream(entries)),
            "cache_index_build");
}

// A device buffer of exactly nbytes from hipMalloc (not the caching
// allocator): the peer exchange exports each store chunk as its own
// allocation, so a peer maps exactly that chunk
torch::Tensor device_alloc(int64_t nbytes, torch::Tensor like) {
  check_dev(like, "like");
  TORCH_CHECK(nbytes > 0, "device_alloc: nbytes > 0");
  c10::DeviceGuard g(like.device());
  void* p = nullptr;
  check_hip(hipMalloc(&p, size_t(nbytes)), "hipMalloc");
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipFree(q); }, like.options().dtype(torch::kUInt8));
}

// IPC: export a device tensor's allocation (handle bytes + the tensor's byte
// offset in it) / map a peer's export as a tensor (closed when it dies)
py::tuple ipc_export(torch::Tensor t) {
  check_dev(t, "t");
  c10::DeviceGuard g(t.device());
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  check_hip(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(t.data_ptr())), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  check_hip(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
  const int64_t off = static_cast<int64_t>(static_cast<const char*>(t.data_ptr()) - static_cast<const char*>(base));
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), off);
}

torch::Tensor ipc_open(py::bytes handle, int64_t offset, std::vector<int64_t> shape, torch::Tensor like) {
  check_dev(like, "like");
  const std::string hb = handle;
  TORCH_CHECK(hb.size() == sizeof(hipIpcMemHandle_t), "ipc_open: bad handle");
  TORCH_CHECK(offset >= 0, "ipc_open: offset >= 0");
  hipIpcMemHandle_t h;
  std::memcpy(&h, hb.data(), sizeof(h));
  c10::DeviceGuard g(like.device());
  void* base = nullptr;
  check_hip(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  void* p = static_cast<char*>(base) + offset;
  return torch::from_blob(p, shape, [base](void*) { (void)hipIpcCloseMemHandle(base); }, like.options());
}

// ---------------------------------------------------------------- K6
// A head's extra logit: fp32 [M], or fp32 [P, >= M] partials summed in order
// (row stride >= M, unit inner stride: the gather-GEMM path's [2, Mp]).
static void check_extra(const torch::Tensor& e, int64_t M) {
  TORCH_CHECK(e.scalar_type() == torch::kFloat32, "extra must be fp32");
  if (e.dim() == 2) {
    TORCH_CHECK(e.size(0) >= 1 && e.size(1) >= M && e.stride(1) == 1 && e.stride(0) >= M,
                "extra partials must be fp32 [P, >= M] with contiguous rows");
  } else {
    TORCH_CHECK(e.numel() == M && e.is_contiguous(), "extra must be fp32 [M]");
  }
}
static int extra_rows(const torch::Tensor& e) { return e.dim() == 2 ? int(e.size(0)) : 1; }
static int64_t extra_stride(const torch::Tensor& e) { return e.dim() == 2 ? e.stride(0) : 0; }

torch::Tensor head(torch::Tensor x, torch::Tensor w, double bias, c10::optional<torch::Tensor> extra, bool sigmoid) {
  check_dev(x, "x");
  check_dev(w, "w");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && x.dim() == 2, "x must be bf16 [M, K]");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8");
  TORCH_CHECK(w.scalar_type() == torch::kFloat32 && w.numel() == K, "w must be fp32 [K]");
  if (extra) {
    check_dev(*extra, "extra");
    check_extra(*extra, M);
  }
  c10::DeviceGuard g(x.device());
  auto out = torch::empty({M}, x.options().dtype(torch::kFloat32));
  check_hip(dtfs::launch_head(x.data_ptr(), K, w.data_ptr<float>(), float(bias),
                              extra ? extra->data_ptr<float>() : nullptr, int(M), int(K), sigmoid ? 2 : 0,
                              out.data_ptr<float>(), cur_stream(x), extra ? extra_rows(*extra) : 1,
                              extra ? extra_stride(*extra) : 0),
            "head");
  return out;
}

// ---------------------------------------------------------------- K4+K6 fused
// Scores [M] fp32 of a fused head kernel: ``out`` (device or pinned host
// memory, which the kernel then writes directly) or a new device tensor.
float* score_out(const torch::Tensor& like, int64_t M, const c10::optional<torch::Tensor>& out, torch::Tensor& y) {
  if (out) {
    TORCH_CHECK(out->scalar_type() == torch::kFloat32 && out->numel() == M && out->is_contiguous(),
                "out must be fp32 [M] contiguous");
    TORCH_CHECK(out->is_cuda() || out->is_pinned(), "out must be on the device or pinned host memory");
    y = *out;
  } else {
    y = torch::empty({M}, like.options().dtype(torch::kFloat32));
  }
  float* yp = y.data_ptr<float>();
  if (!y.is_cuda()) {
    // pinned host allocations are mapped at the same virtual address on ROCm;
    // prefer the runtime's answer when it has one
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, yp, 0) == hipSuccess && dp)
      yp = static_cast<float*>(dp);
    else
      (void)hipGetLastError();
  }
  return yp;
}

torch::Tensor gemm_head(torch::Tensor A, torch::Tensor W, torch::Tensor bias, int64_t act, torch::Tensor hw,
                        double hbias, c10::optional<torch::Tensor> extra, bool sigmoid,
                        c10::optional<torch::Tensor> out) {
  check_dev(A, "A");
  check_dev(W, "W");
  check_dev(bias, "bias");
  check_dev(hw, "hw");
  check_same_dev(A, W, "W");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && W.scalar_type() == torch::kBFloat16, "A, W must be bf16");
  TORCH_CHECK(A.dim() == 2 && W.dim() == 2 && A.size(1) == W.size(1), "A [M, K], W [N, K]");
  TORCH_CHECK(A.is_contiguous() && W.is_contiguous(), "A, W must be contiguous");
  const int64_t M = A.size(0), K = A.size(1), N = W.size(0);
  TORCH_CHECK(K % 64 == 0, "gemm_head needs K % 64 == 0");
  TORCH_CHECK(N > 0 && N <= 256, "gemm_head needs 0 < N <= 256");
  TORCH_CHECK(act == 0 || act == 1, "act must be 0 (none) or 1 (relu)");
  TORCH_CHECK(bias.scalar_type() == torch::kFloat32 && bias.numel() == N, "bias must be fp32 [N]");
  TORCH_CHECK(hw.scalar_type() == torch::kFloat32 && hw.numel() == N, "hw must be fp32 [N]");
  if (extra) {
    check_dev(*extra, "extra");
    check_extra(*extra, M);
  }
  c10::DeviceGuard g(A.device());
  torch::Tensor y;
  float* yp = score_out(A, M, out, y);
  check_hip(dtfs::launch_gemm_head(A.data_ptr(), K, W.data_ptr(), K, bias.data_ptr<float>(), int(act),
                                   hw.data_ptr<float>(), float(hbias), extra ? extra->data_ptr<float>() : nullptr,
                                   sigmoid ? 2 : 0, yp, int(M), int(N), int(K), cur_stream(A),
                                   extra ? extra_rows(*extra) : 1, extra ? extra_stride(*extra) : 0),
            "gemm_head");
  return y;
}

// K4 + K4 + K6: the two-layer MLP tail + head in one launch (mlp_tail.hip).
// W2p / W3p hold the weights in MFMA fragment order (ops.pack_bfrag).
torch::Tensor mlp_tail(torch::Tensor X, torch::Tensor W2p, torch::Tensor b2, int64_t act2, torch::Tensor W3p,
                       torch::Tensor b3, int64_t act3, torch::Tensor hw, double hbias,
                       c10::optional<torch::Tensor> extra, bool sigmoid, c10::optional<torch::Tensor> out) {
  for (auto* t : {&X, &W2p, &b2, &W3p, &b3, &hw}) check_dev(*t, "mlp_tail operand");
  check_same_dev(X, W2p, "W2p");
  check_same_dev(X, W3p, "W3p");
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && X.dim() == 2 && X.stride(1) == 1, "X must be bf16 [M, K1] rows");
  TORCH_CHECK(W2p.scalar_type() == torch::kBFloat16 && W3p.scalar_type() == torch::kBFloat16 && W2p.is_contiguous() &&
                  W3p.is_contiguous(),
              "W2p, W3p must be contiguous bf16 (pack_bfrag)");
  const int64_t M = X.size(0), K1 = X.size(1), N2 = b2.numel(), N3 = b3.numel();
  TORCH_CHECK(N2 == 512 && N3 == 256, "mlp_tail covers N2 = 512, N3 = 256");
  TORCH_CHECK(K1 == 1024, "mlp_tail covers K1 = 1024");
  TORCH_CHECK(K1 % 128 == 0 && X.stride(0) % 8 == 0, "mlp_tail needs K1 % 128 == 0 and 16-byte rows");
  TORCH_CHECK(W2p.numel() == N2 * K1 && W3p.numel() == N3 * N2, "packed weight sizes");
  TORCH_CHECK(b2.scalar_type() == torch::kFloat32 && b3.scalar_type() == torch::kFloat32 &&
                  hw.scalar_type() == torch::kFloat32 && hw.numel() == N3,
              "b2, b3, hw must be fp32 [N2], [N3], [N3]");
  TORCH_CHECK((act2 == 0 || act2 == 1) && (act3 == 0 || act3 == 1), "act must be 0 (none) or 1 (relu)");
  if (extra) {
    check_dev(*extra, "extra");
    check_extra(*extra, M);
  }
  c10::DeviceGuard g(X.device());
  torch::Tensor y;
  float* yp = score_out(X, M, out, y);
  check_hip(dtfs::launch_mlp_tail(X.data_ptr(), X.stride(0), int(M), int(K1), W2p.data_ptr(), b2.data_ptr<float>(),
                                  int(act2), int(N2), W3p.data_ptr(), b3.data_ptr<float>(), int(act3), int(N3),
                                  hw.data_ptr<float>(), float(hbias), extra ? extra->data_ptr<float>() : nullptr,
                                  extra ? extra_rows(*extra) : 0, extra ? extra_stride(*extra) : 0, sigmoid ? 2 : 0,
                                  yp, cur_stream(X)),
            "mlp_tail");
  return y;
}

// K1 + K2 + K4 x 3 + K6: the whole DeepFM / Wide&Deep tower in one launch,
// the resolve pass included (gather_mlp.hip): 64 rows x all 1024 h1 columns per
// workgroup, h1 / h2 kept in LDS. W1p / W2p / W3p: ops.pack_frag32 of the three
// weights. ``fm``: add the second-order FM term of each row (DeepFM). Returns
// the scores (fp32 [B], or ``out``: device or pinned host memory).
torch::Tensor gather_mlp(torch::Tensor table, c10::optional<torch::Tensor> lin, c10::optional<torch::Tensor> arena,
                         c10::optional<torch::Tensor> ids, c10::optional<torch::Tensor> wts, int64_t B, int64_t F,
                         int64_t modulo, double bias, torch::Tensor W1p, torch::Tensor b1, torch::Tensor W2p,
                         torch::Tensor b2, int64_t act2, torch::Tensor W3p, torch::Tensor b3, int64_t act3,
                         torch::Tensor hw, double hbias, bool fm, bool sigmoid, c10::optional<torch::Tensor> out) {
  check_dev(table, "table");
  for (auto* t : {&W1p, &b1, &W2p, &b2, &W3p, &b3, &hw}) {
    check_dev(*t, "gather_mlp operand");
    check_same_dev(table, *t, "gather_mlp operand");
  }
  TORCH_CHECK(table.scalar_type() == torch::kBFloat16 && table.dim() == 2 && table.size(1) == 64 &&
                  table.is_contiguous(),
              "gather_mlp: table must be contiguous bf16 [V, 64]");
  const int64_t V = table.size(0);
  TORCH_CHECK(F >= 1 && F <= 64, "gather_mlp handles 1..64 fields");
  TORCH_CHECK(modulo > 0 && modulo <= V, "modulo must be in (0, table rows]");
  for (auto* t : {&W1p, &W2p, &W3p})
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->is_contiguous(), "W1p / W2p / W3p: contiguous bf16 (pack_frag32)");
  TORCH_CHECK(b1.scalar_type() == torch::kFloat32 && b1.numel() == 1024 && b2.scalar_type() == torch::kFloat32 &&
                  b2.numel() == 512 && b3.scalar_type() == torch::kFloat32 && b3.numel() == 256 &&
                  hw.scalar_type() == torch::kFloat32 && hw.numel() == 256,
              "gather_mlp covers 64F -> 1024 -> 512 -> 256 -> 1 (fp32 biases / head weights)");
  TORCH_CHECK(W1p.numel() == 1024 * 64 * F && W2p.numel() == 512 * 1024 && W3p.numel() == 256 * 512,
              "packed weight sizes");
  TORCH_CHECK((act2 == 0 || act2 == 1) && (act3 == 0 || act3 == 1), "act must be 0 (none) or 1 (relu)");
  TORCH_CHECK(B >= 0 && B < (int64_t(1) << 31), "gather_mlp: row count");
  if (lin) {
    check_dev(*lin, "lin");
    TORCH_CHECK(lin->scalar_type() == torch::kFloat32 && lin->numel() == V, "lin must be fp32 [V]");
  }
  TORCH_CHECK(dtfs::gather_mlp_ok((B + 63) / 64 * 64, 1024, int(64 * F), 512, 256, int(F), V),
              "gather_mlp: shape outside the kernel's range");
  dtfs::EmbedArgs a;
  embed_gemm_inputs(table, arena, ids, wts, B, F, a);
  a.table = table.data_ptr();
  a.lin = lin ? lin->data_ptr<float>() : nullptr;
  a.B = int(B);
  a.F = int(F);
  a.D = 64;
  a.V = V;
  a.modulo = modulo;
  a.bias = float(bias);
  c10::DeviceGuard g(table.device());
  torch::Tensor y;
  float* yp = score_out(table, B, out, y);
  if (B == 0) return y;
  check_hip(dtfs::launch_gather_mlp(a, W1p.data_ptr(), b1.data_ptr<float>(), W2p.data_ptr(), b2.data_ptr<float>(),
                                    int(act2), W3p.data_ptr(), b3.data_ptr<float>(), int(act3), hw.data_ptr<float>(),
                                    float(hbias), fm, sigmoid ? 2 : 0, yp, cur_stream(table)),
            "gather_mlp");
  return y;
}

// ---------------------------------------------------------------- K0 ingest
void unpack_arena(torch::Tensor arena, torch::Tensor packed, int64_t fields, int64_t narrow_modulo) {
  check_dev(arena, "arena");
  check_dev(packed, "packed");
  check_same_dev(arena, packed, "packed");
  TORCH_CHECK(arena.scalar_type() == torch::kUInt8 && arena.numel() > dtfs::kArenaPayloadOff, "arena: uint8 [cap]");
  TORCH_CHECK(packed.scalar_type() == torch::kInt64 && packed.dim() == 2, "packed must be int64 [B, W]");
  TORCH_CHECK(packed.size(1) * 8 >= (narrow_modulo > 0 ? 8 : 12) * fields, "packed rows too narrow for the field count");
  TORCH_CHECK(narrow_modulo >= 0 && narrow_modulo < (int64_t(1) << 31), "narrow_modulo must fit int32 rows");
  c10::DeviceGuard g(arena.device());
  // descriptor offsets come from the (validated) host parse of this arena; the
  // kernel additionally bounds n_req by the descriptor capacity
  check_hip(dtfs::launch_unpack_arena(arena.data_ptr(), packed.data_ptr<int64_t>(), int(packed.size(0)), int(fields),
                                      int(packed.size(1)), dtfs::kArenaMaxRequests, cur_stream(arena), narrow_modulo),
            "unpack_arena");
}

void arena_varint_decode(torch::Tensor arena, int64_t blocks) {
  check_dev(arena, "arena");
  TORCH_CHECK(arena.scalar_type() == torch::kUInt8 && arena.numel() > dtfs::kArenaPayloadOff, "arena: uint8 [cap]");
  c10::DeviceGuard g(arena.device());
  // chunk offsets come from the validated host build of this arena
  check_hip(dtfs::launch_arena_varint(arena.data_ptr(), int(blocks), cur_stream(arena)), "arena_varint_decode");
}

void pull_host(torch::Tensor dst, torch::Tensor src, int64_t nbytes, int64_t blocks) {
  check_dev(dst, "dst");
  TORCH_CHECK(src.device().is_cpu() && src.is_pinned(), "src must be pinned host memory");
  TORCH_CHECK(nbytes >= 0 && nbytes <= dst.nbytes() && nbytes <= src.nbytes(), "nbytes out of range");
  c10::DeviceGuard g(dst.device());
  check_hip(dtfs::launch_pull_host(dst.data_ptr(), src.data_ptr(), nbytes, int(blocks), cur_stream(dst)), "pull_host");
}

// ---------------------------------------------------------------- fp8
torch::Tensor dense_pad(torch::Tensor x, int64_t n, int64_t K) {
  TORCH_CHECK(x.is_cuda(), "x must be a GPU tensor");  // a row view of packed request rows
  TORCH_CHECK(x.scalar_type() == torch::kFloat32 && x.dim() == 2 && x.stride(1) == 1 && x.stride(0) >= n &&
                  x.size(1) >= n,
              "x must be fp32 [M, >= n] with contiguous rows");
  TORCH_CHECK(K % 8 == 0 && n >= 0 && n <= K, "K % 8 == 0, 0 <= n <= K");
  c10::DeviceGuard g(x.device());
  auto y = torch::empty({x.size(0), K}, x.options().dtype(torch::kBFloat16));
  check_hip(dtfs::launch_dense_pad(x.data_ptr<float>(), x.stride(0), int(x.size(0)), int(n), y.data_ptr(), int(K),
                                   cur_stream(x)),
            "dense_pad");
  return y;
}

std::vector<torch::Tensor> quant_rows_fp8(torch::Tensor x, int64_t k_pad) {
  check_dev(x, "x");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && x.dim() == 2, "x must be bf16 [M, K]");
  TORCH_CHECK(x.stride(1) == 1, "x rows must be contiguous");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(K % 8 == 0 && K <= 4096, "K must be a multiple of 8 and <= 4096");
  TORCH_CHECK(k_pad >= 1 && k_pad <= 256, "k_pad must be in [1, 256]");
  const int64_t Kq = (K + k_pad - 1) / k_pad * k_pad;
  TORCH_CHECK(Kq % 16 == 0, "padded K must be a multiple of 16");
  c10::DeviceGuard g(x.device());
  auto q = torch::empty({M, Kq}, x.options().dtype(torch::kFloat8_e4m3fn));
  auto s = torch::empty({M}, x.options().dtype(torch::kFloat32));
  check_hip(dtfs::launch_quant_rows_fp8(x.data_ptr(), x.stride(0), int(M), int(K), q.data_ptr(), Kq,
                                        s.data_ptr<float>(), cur_stream(x), int(Kq)),
            "quant_rows_fp8");
  return {q, s};
}

// z = x0 * y + xl (+ fp8 quantisation of z, + head dot): the split DCN-v2 cross layer's combine pass
std::vector<torch::Tensor> cross_combine(torch::Tensor y, torch::Tensor x0, torch::Tensor xl, bool want_z,
                                         int64_t k_pad, c10::optional<torch::Tensor> head_w) {
  check_dev(y, "y");
  for (auto* t : {&y, &x0, &xl})
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->dim() == 2 && t->is_contiguous() &&
                    t->sizes() == y.sizes() && t->device() == y.device(),
                "y, x0, xl must be contiguous bf16 [M, N] on one device");
  const int64_t M = y.size(0), N = y.size(1);
  TORCH_CHECK(N % 8 == 0 && N <= 4096, "N must be a multiple of 8 and <= 4096");
  TORCH_CHECK(k_pad >= 0 && k_pad <= 256, "k_pad must be in [0, 256] (0 = no quantisation)");
  c10::DeviceGuard g(y.device());
  torch::Tensor z, q, s, dot;
  if (want_z) z = torch::empty({M, N}, y.options());
  int64_t Kq = 0;
  if (k_pad > 0) {
    Kq = (N + k_pad - 1) / k_pad * k_pad;
    TORCH_CHECK(Kq % 16 == 0, "padded K must be a multiple of 16");
    q = torch::empty({M, Kq}, y.options().dtype(torch::kFloat8_e4m3fn));
    s = torch::empty({M}, y.options().dtype(torch::kFloat32));
  }
  const float* hw = nullptr;
  if (head_w && head_w->defined()) {
    TORCH_CHECK(head_w->scalar_type() == torch::kFloat32 && head_w->numel() == N && head_w->is_contiguous() &&
                    head_w->device() == y.device(),
                "head_w must be fp32 [N] on y's device");
    hw = head_w->data_ptr<float>();
    dot = torch::empty({M}, y.options().dtype(torch::kFloat32));
  }
  TORCH_CHECK(want_z || k_pad > 0 || hw, "nothing to produce");
  check_hip(dtfs::launch_cross_combine(y.data_ptr(), x0.data_ptr(), xl.data_ptr(), N, int(M), int(N),
                                       want_z ? z.data_ptr() : nullptr, N, k_pad > 0 ? q.data_ptr() : nullptr, Kq,
                                       k_pad > 0 ? s.data_ptr<float>() : nullptr, int(Kq), hw,
                                       hw ? dot.data_ptr<float>() : nullptr, cur_stream(y)),
            "cross_combine");
  return {z, q, s, dot};
}

// One DCN-v2 cross layer, fp8 GEMM + LDS-staged cross epilogue in one launch:
// z = bf16(x0 * bf16(q W^T * sx * sw + b) + xl) (want_z) and / or the cross
// logit as partials dot[tn, m] = z[m, 256 tn .. +256] . head_w (the head sums
// them). Same rounding as linear_fp8 (plain) + cross_combine.
std::vector<torch::Tensor> cross_gemm_fp8(torch::Tensor q, torch::Tensor sx, torch::Tensor Wq, torch::Tensor sw,
                                          c10::optional<torch::Tensor> bias, torch::Tensor x0, torch::Tensor xl,
                                          bool want_z, c10::optional<torch::Tensor> head_w) {
  check_dev(q, "q");
  check_same_dev(q, Wq, "Wq");
  TORCH_CHECK(q.scalar_type() == torch::kFloat8_e4m3fn && Wq.scalar_type() == torch::kFloat8_e4m3fn && q.dim() == 2 &&
                  Wq.dim() == 2 && q.is_contiguous() && Wq.is_contiguous(),
              "q [M, K] and Wq [N, K] must be contiguous e4m3");
  const int64_t M = q.size(0), K = q.size(1), N = Wq.size(0);
  TORCH_CHECK(Wq.size(1) == K && K % 128 == 0, "K mismatch or K % 128 != 0: q ", q.sizes(), " Wq ", Wq.sizes());
  TORCH_CHECK(N % 8 == 0 && M < (int64_t(1) << 31), "N must be a multiple of 8");
  for (auto* t : {&sx, &sw}) {
    check_same_dev(q, *t, "scales");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->is_contiguous(), "scales must be contiguous fp32");
  }
  TORCH_CHECK(sx.numel() == M && sw.numel() == N, "sx [M], sw [N]");
  if (bias) {
    check_same_dev(q, *bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == N && bias->is_contiguous(),
                "bias must be fp32 [N]");
  }
  for (auto* t : {&x0, &xl}) {
    check_same_dev(q, *t, "x0/xl");
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->dim() == 2 && t->size(0) == M && t->size(1) == N &&
                    t->is_contiguous(),
                "x0/xl must be contiguous bf16 [M, N]");
  }
  const float* hw = nullptr;
  if (head_w && head_w->defined()) {
    check_same_dev(q, *head_w, "head_w");
    TORCH_CHECK(head_w->scalar_type() == torch::kFloat32 && head_w->numel() == N && head_w->is_contiguous(),
                "head_w must be fp32 [N]");
    hw = head_w->data_ptr<float>();
  }
  TORCH_CHECK(want_z || hw, "nothing to produce");
  c10::DeviceGuard g(q.device());
  const int64_t tiles_n = (N + 255) / 256;
  torch::Tensor z, dot;
  if (want_z) z = torch::empty({M, N}, x0.options());
  if (hw) dot = torch::empty({tiles_n, M}, x0.options().dtype(torch::kFloat32));
  dtfs::CrossGemmArgs a;
  a.A = q.data_ptr();
  a.lda = K;
  a.W = Wq.data_ptr();
  a.ldw = K;
  a.bias = bias ? bias->data_ptr<float>() : nullptr;
  a.sa = sx.data_ptr<float>();
  a.sw = sw.data_ptr<float>();
  a.Z = want_z ? z.data_ptr() : nullptr;
  a.ldz = N;
  a.X0 = x0.data_ptr();
  a.XL = xl.data_ptr();
  a.ldx = N;
  a.hw = hw;
  a.dot = hw ? dot.data_ptr<float>() : nullptr;
  a.ldd = M;
  a.M = int(M);
  a.N = int(N);
  a.K = int(K);
  check_hip(dtfs::launch_cross_gemm_fp8(a, cur_stream(q)), "cross_gemm_fp8");
  return {z, dot};
}

// ---------------------------------------------------------------- K7
std::vector<torch::Tensor> sort_scores(torch::Tensor s, bool descending, int64_t k) {
  check_dev(s, "scores");
  TORCH_CHECK(s.scalar_type() == torch::kFloat32 && s.dim() == 1, "scores must be fp32 [N]");
  const int64_t n = s.numel();
  TORCH_CHECK(n <= dtfs::sort_max_elems(), "sort kernel handles at most ", dtfs::sort_max_elems(), " scores");
  if (k < 0 || k > n) k = n;
  c10::DeviceGuard g(s.device());
  auto out = torch::empty({k}, s.options());
  auto perm = torch::empty({k}, s.options().dtype(torch::kInt64));
  check_hip(dtfs::launch_sort_scores(s.data_ptr<float>(), int(n), descending, out.data_ptr<float>(),
                                     perm.data_ptr<int64_t>(), int(k), cur_stream(s)),
            "sort_scores");
  return {out, perm};
}

// ---------------------------------------------------------------- fan-out step
// Validates the device/host buffers of one fan-out step (everything but the
// per-step H2D source) and computes the per-peer message sizes.
dtfs::runtime::FanoutStep make_fanout_step(torch::Tensor h2d_dst, uintptr_t ingress_exec, dtfs::comm::RcclComm& cin,
                                           int mode, torch::Tensor send, torch::Tensor recv, uintptr_t forward_exec,
                                           dtfs::comm::RcclComm& cout, torch::Tensor scores, torch::Tensor back,
                                           torch::Tensor h_out, int64_t d2h_bytes) {
  TORCH_CHECK(mode == 0 || mode == 1, "mode: 0 all-to-all, 1 scatter/gather");
  TORCH_CHECK(cin.nranks() == cout.nranks() && cin.rank() == cout.rank(), "communicator mismatch");
  const int W = cin.nranks();
  for (auto* t : {&h2d_dst, &send, &recv, &scores, &back})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous(), "fan-out buffers must be contiguous GPU tensors");
  TORCH_CHECK(h_out.device().is_cpu() && h_out.is_pinned(), "h_out must be pinned host memory");
  // all-to-all: send/recv (and scores/back) are this rank's B rows, B/W to /
  // from each peer. scatter/gather: recv/scores are this rank's B rows; the
  // root's send/back hold W x B.
  size_t in_bytes, out_bytes;
  if (mode == 0) {
    TORCH_CHECK(send.nbytes() == recv.nbytes() && recv.nbytes() % W == 0,
                "all-to-all: send and recv must match and split evenly over the ranks");
    TORCH_CHECK(back.nbytes() == scores.nbytes() && scores.nbytes() % W == 0,
                "all-to-all: scores and back must match and split evenly over the ranks");
    in_bytes = recv.nbytes() / W;
    out_bytes = scores.nbytes() / W;
  } else {
    in_bytes = recv.nbytes();
    out_bytes = scores.nbytes();
    if (cin.rank() == 0) {
      TORCH_CHECK(send.nbytes() >= in_bytes * W, "scatter: root send smaller than world x recv");
      TORCH_CHECK(back.nbytes() >= out_bytes * W, "gather: root back smaller than world x scores");
    }
  }
  TORCH_CHECK(d2h_bytes >= 0 && size_t(d2h_bytes) <= back.nbytes() && size_t(d2h_bytes) <= h_out.nbytes(),
              "d2h_bytes out of range");
  TORCH_CHECK(forward_exec != 0, "null forward graph");
  dtfs::runtime::FanoutStep s;
  s.h2d_dst = h2d_dst.data_ptr();
  s.ingress = reinterpret_cast<hipGraphExec_t>(ingress_exec);
  s.cin = &cin;
  s.mode = mode;
  s.send = send.data_ptr();
  s.recv = recv.data_ptr();
  s.in_bytes = in_bytes;
  s.forward = reinterpret_cast<hipGraphExec_t>(forward_exec);
  s.cout = &cout;
  s.scores = scores.data_ptr();
  s.back = back.data_ptr();
  s.out_bytes = out_bytes;
  s.h_out = h_out.data_ptr();
  s.d2h_bytes = size_t(d2h_bytes);
  return s;
}

// A programmed step (StepRunner::launch_program) from its Python description:
// {"h2d_dst": tensor, "h2d_lane": int, "ops": [dict, ...]} with op dicts
//   {"kind": "kernels", "lane": l, "seq": KernelSequence | None, "graph_exec": int}
//   {"kind": "alltoall" | "allgather" | "reduce_scatter", "lane": l, "comm": RcclComm, "send": t, "recv": t}
//   {"kind": "record" | "wait" | "wait_prev", "lane": l, "event": k}
// Message sizes come from the tensors (validated here, once).
dtfs::runtime::StepProgram program_from(const py::dict& d, std::vector<py::object>* keep) {
  keep->push_back(d);
  dtfs::runtime::StepProgram p;
  torch::Tensor dst = d["h2d_dst"].cast<torch::Tensor>();
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "h2d_dst must be a contiguous GPU tensor");
  p.h2d_dst = dst.data_ptr();
  p.h2d_lane = d.contains("h2d_lane") ? d["h2d_lane"].cast<int>() : 1;
  for (auto item : d["ops"].cast<py::list>()) {
    py::dict o = item.cast<py::dict>();
    dtfs::runtime::ProgOp op;
    const std::string kind = o["kind"].cast<std::string>();
    op.lane = o.contains("lane") ? o["lane"].cast<int>() : 0;
    if (kind == "kernels") {
      op.kind = dtfs::runtime::ProgOp::kKernels;
      if (o.contains("seq") && !o["seq"].is_none()) op.seq = &o["seq"].cast<dtfs::runtime::KernelSequence&>();
      if (o.contains("graph_exec")) op.graph = reinterpret_cast<hipGraphExec_t>(o["graph_exec"].cast<uintptr_t>());
    } else if (kind == "record" || kind == "wait" || kind == "wait_prev") {
      op.kind = kind == "record" ? dtfs::runtime::ProgOp::kRecord
                : kind == "wait" ? dtfs::runtime::ProgOp::kWait
                                 : dtfs::runtime::ProgOp::kWaitPrev;
      op.event = o["event"].cast<int>();
    } else {
      auto& c = o["comm"].cast<dtfs::comm::RcclComm&>();
      torch::Tensor send = o["send"].cast<torch::Tensor>(), recv = o["recv"].cast<torch::Tensor>();
      TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                  "collective buffers must be contiguous GPU tensors");
      const size_t W = size_t(c.nranks());
      op.comm = &c;
      op.send = send.data_ptr();
      op.recv = recv.data_ptr();
      if (kind == "alltoall") {
        TORCH_CHECK(send.nbytes() == recv.nbytes() && send.nbytes() % W == 0,
                    "all-to-all: send and recv must match and split evenly over the ranks");
        op.kind = dtfs::runtime::ProgOp::kAllToAll;
        op.bytes = send.nbytes() / W;
      } else if (kind == "allgather") {
        TORCH_CHECK(recv.nbytes() == send.nbytes() * W, "all-gather: recv must be world x send");
        op.kind = dtfs::runtime::ProgOp::kAllGather;
        op.bytes = send.nbytes();
      } else if (kind == "reduce_scatter") {
        TORCH_CHECK(send.scalar_type() == torch::kBFloat16 && recv.scalar_type() == torch::kBFloat16,
                    "reduce-scatter buffers must be bf16");
        TORCH_CHECK(size_t(send.numel()) == size_t(recv.numel()) * W, "reduce-scatter: send must be world x recv");
        op.kind = dtfs::runtime::ProgOp::kReduceScatter;
        op.bytes = size_t(recv.numel());
      } else {
        TORCH_CHECK(false, "unknown program op kind ", kind);
      }
    }
    p.ops.push_back(op);
  }
  try {
    p.validate();
  } catch (const std::invalid_argument& e) {
    TORCH_CHECK(false, e.what());
  }
  return p;
}

// One native loop slot from its Python description (FanoutEngine.loop_slots).
dtfs::runtime::LoopSlot loop_slot_from(const py::dict& d, std::vector<py::object>* keep) {
  keep->push_back(d);
  dtfs::runtime::LoopSlot s;
  torch::Tensor h_out = d["h_out"].cast<torch::Tensor>();
  TORCH_CHECK(h_out.device().is_cpu() && h_out.is_pinned() && h_out.scalar_type() == torch::kFloat32 &&
                  h_out.is_contiguous(),
              "h_out must be a pinned contiguous fp32 tensor");
  s.h_out = h_out.data_ptr<float>();
  s.h_out_len = h_out.numel();
  torch::Tensor dst = d["h2d_dst"].cast<torch::Tensor>();
  TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "h2d_dst must be a contiguous GPU tensor");
  if (d.contains("program") && !d["program"].is_none()) {
    s.program = true;
    s.prog = program_from(d["program"].cast<py::dict>(), keep);
    s.h2d_cap = int64_t(dst.nbytes());
    TORCH_CHECK(s.prog.h2d_dst == dst.data_ptr(), "program h2d_dst must be the slot's h2d_dst");
  } else if (d.contains("fanout") && d["fanout"].cast<bool>()) {
    s.fanout = true;
    s.fan = make_fanout_step(dst, d["ingress_exec"].cast<uintptr_t>(), d["cin"].cast<dtfs::comm::RcclComm&>(),
                             d["mode"].cast<int>(), d["send"].cast<torch::Tensor>(), d["recv"].cast<torch::Tensor>(),
                             d["forward_exec"].cast<uintptr_t>(), d["cout"].cast<dtfs::comm::RcclComm&>(),
                             d["scores"].cast<torch::Tensor>(), d["back"].cast<torch::Tensor>(), h_out,
                             d["d2h_bytes"].cast<int64_t>());
    if (d.contains("forward_seq") && !d["forward_seq"].is_none())
      s.fan.forward_seq = &d["forward_seq"].cast<dtfs::runtime::KernelSequence&>();
    if (d.contains("ingress_seq") && !d["ingress_seq"].is_none())
      s.fan.ingress_seq = &d["ingress_seq"].cast<dtfs::runtime::KernelSequence&>();
    if (d.contains("resolve_exec") && !d["resolve_exec"].is_none())
      s.fan.resolve = reinterpret_cast<hipGraphExec_t>(d["resolve_exec"].cast<uintptr_t>());
    if (d.contains("resolve_seq") && !d["resolve_seq"].is_none())
      s.fan.resolve_seq = &d["resolve_seq"].cast<dtfs::runtime::KernelSequence&>();
  } else {
    s.h2d_dst = dst.data_ptr();
    s.h2d_cap = int64_t(dst.nbytes());
    if (d.contains("seq") && !d["seq"].is_none()) s.seq = &d["seq"].cast<dtfs::runtime::KernelSequence&>();
    if (d.contains("graph_exec")) s.graph = reinterpret_cast<hipGraphExec_t>(d["graph_exec"].cast<uintptr_t>());
    TORCH_CHECK(s.graph != nullptr || s.seq != nullptr, "slot needs a step graph or kernel sequence");
  }
  return s;
}

// ---------------------------------------------------------------- live server (GPU backend)
// The device side of a GPU live server: the StepRunner plus, per bucket and
// slot, the step to launch (direct kernel launches of the captured step, its
// graph, or the fan-out step with its RCCL communicators).
// One shared-scatter step of this rank (runtime/shared_scatter.h): rank 0
// publishes the plan over its built shared arena, every rank copies only its
// share (copy stream, its own PCIe link) into `dst` and launches the local step
// on it; the step's head writes the rank's scores into rank 0's shared output.
// Returns the step index.
uint64_t scatter_step(dtfs::runtime::StepRunner& r, dtfs::runtime::SharedScatter& sc, int slot, int64_t rows_per_rank,
                      const uint8_t* arena, void* dst, int64_t dst_cap, const dtfs::runtime::KernelSequence* seq,
                      hipGraphExec_t graph, int64_t timeout_us) {
  const uint64_t k = sc.begin_step();
  if (sc.rank() == 0) {
    const int ai = arena ? sc.arena_index(arena) : -1;
    if (ai < 0) throw std::runtime_error("shared scatter: rank 0's batch is not in a shared arena");
    sc.publish_plan(k, ai, rows_per_rank);
  }
  dtfs::runtime::RankShare mine;
  int ai = -1;
  if (!sc.wait_plan(k, timeout_us, &mine, &ai))
    throw std::runtime_error("shared scatter: no plan for step " + std::to_string(k) + " from rank 0");
  const auto copies = dtfs::runtime::share_copies(sc.arena(ai), mine, sc.stage(slot));
  int64_t n = 0;
  for (const auto& c : copies) {
    if (c.dst_off < 0 || c.dst_off + c.n > dst_cap) throw std::runtime_error("shared scatter: share outside the device arena");
    n += c.n;
  }
  sc.add_h2d(n);
  r.launch_copies(slot, dst, copies, seq, graph, true);
  return k;
}

// Wait for step k on `slot`: this rank's step, then (rank 0) every rank's share.
bool scatter_wait(dtfs::runtime::StepRunner& r, dtfs::runtime::SharedScatter& sc, int slot, uint64_t k,
                  int64_t timeout_us, const std::vector<dtfs::comm::RcclComm*>& comms, std::string* err) {
  if (!r.wait_for(slot, timeout_us, comms, err)) return false;
  sc.mark_done(k);
  if (sc.rank() != 0) return true;
  if (!sc.wait_done(k, timeout_us, err)) return false;
  sc.compact_scores(k, slot);
  return true;
}

class GpuBackend : public dtfs::runtime::StepBackend {
 public:
  GpuBackend(dtfs::runtime::StepRunner* runner, std::vector<int64_t> buckets,
             std::vector<std::vector<dtfs::runtime::LoopSlot>> slots)
      : runner_(runner), buckets_(std::move(buckets)), slots_(std::move(slots)) {
    TORCH_CHECK(!slots_.empty() && slots_.size() == buckets_.size(), "one slot list per bucket");
    const size_t S = slots_[0].size();
    TORCH_CHECK(S >= 1 && int(S) <= runner_->slots(), "slot count must be in [1, runner slots]");
    for (const auto& v : slots_) TORCH_CHECK(v.size() == S, "every bucket needs the same number of slots");
    auto add = [&](dtfs::comm::RcclComm* c) {
      if (c && std::find(comms_.begin(), comms_.end(), c) == comms_.end()) comms_.push_back(c);
    };
    for (const auto& v : slots_)
      for (const auto& s : v) {
        if (s.fanout)
          for (auto* c : {s.fan.cin, s.fan.cout}) add(c);
        if (s.program)
          for (const auto& o : s.prog.ops) add(o.comm);
      }
  }
  int slots() const override { return int(slots_[0].size()); }
  const std::vector<int64_t>& buckets() const override { return buckets_; }
  // shared-scatter mode: every local-kind slot's step runs on this rank's
  // share of rank 0's batch; share_rows[b] = rows per rank of bucket b
  void set_scatter(dtfs::runtime::SharedScatter* sc, std::vector<int64_t> share_rows, int64_t timeout_us) {
    TORCH_CHECK(share_rows.size() == buckets_.size(), "shared scatter: one share row count per bucket");
    TORCH_CHECK(slots() <= dtfs::runtime::kScatterMaxSlots && slots() <= sc->slots(), "shared scatter: too many slots");
    sc_ = sc;
    share_rows_ = std::move(share_rows);
    slot_step_.assign(size_t(slots()), 0);
    timeout_us_ = timeout_us;
  }
  void launch(int slot, int b, const uint8_t* arena, const dtfs::runtime::ArenaBatch& batch) override {
    const auto& s = slots_[size_t(b)][size_t(slot)];
    if (sc_ && !s.program && !s.fanout) {
      slot_step_[size_t(slot)] = scatter_step(*runner_, *sc_, slot, share_rows_[size_t(b)], arena, s.h2d_dst,
                                              s.h2d_cap, s.seq, s.graph, timeout_us_);
      return;
    }
    // the header + descriptors always travel, so an empty (lockstep) step
    // sees zero rows instead of the slot's previous batch
    const int64_t nbytes = batch.used_bytes;
    if (s.program) {
      if (nbytes > s.h2d_cap) throw std::runtime_error("batch larger than the device arena");
      runner_->launch_program(slot, s.prog, arena, nbytes, batch.n_gpu_varint == 0);
    } else if (s.fanout) {
      dtfs::runtime::FanoutStep f = s.fan;
      f.h2d_src = arena;
      f.h2d_bytes = nbytes;
      f.skip_varint = batch.n_gpu_varint == 0;
      runner_->launch_fanout(slot, f);
    } else {
      if (nbytes > s.h2d_cap) throw std::runtime_error("batch larger than the device arena");
      if (s.seq) runner_->launch_seq(slot, s.h2d_dst, arena, nbytes, s.seq, batch.n_gpu_varint == 0);
      else runner_->launch(slot, s.h2d_dst, arena, nbytes, s.graph);
    }
  }
  bool wait(int slot, int64_t timeout_us, std::string* err) override {
    if (sc_) return scatter_wait(*runner_, *sc_, slot, slot_step_[size_t(slot)], timeout_us, comms_, err);
    return runner_->wait_for(slot, timeout_us, comms_, err);
  }
  const float* scores(int slot, int b) const override { return slots_[size_t(b)][size_t(slot)].h_out; }
  int64_t scores_len(int slot, int b) const override { return slots_[size_t(b)][size_t(slot)].h_out_len; }
  void abort() override {
    for (auto* c : comms_)
      if (c && !c->aborted()) c->abort();
  }

 private:
  dtfs::runtime::StepRunner* runner_;
  std::vector<int64_t> buckets_;
  std::vector<std::vector<dtfs::runtime::LoopSlot>> slots_;  // [bucket][slot]
  std::vector<dtfs::comm::RcclComm*> comms_;
  dtfs::runtime::SharedScatter* sc_ = nullptr;
  std::vector<int64_t> share_rows_;
  std::vector<uint64_t> slot_step_;  // step index of each slot's last launch (launcher writes, completer reads)
  int64_t timeout_us_ = 10'000'000;
};

struct PyGpuLive {
  std::vector<py::object> keep;
  std::unique_ptr<GpuBackend> backend;
  std::unique_ptr<dtfs::runtime::LiveServer> srv;
  ~PyGpuLive() {
    py::gil_scoped_release nogil;
    srv.reset();
  }
};

// buckets: [(rows, [slot dict per slot]), ...] ascending.
PyGpuLive* make_gpu_live(py::object runner_obj, py::dict cfg, py::list buckets, py::list arenas,
                         py::object control, py::object scatter, py::object share_rows) {
  auto* p = new PyGpuLive();
  dtfs::runtime::StepControl* ctl = dtfs_live::control_from(control, &p->keep);
  p->keep.push_back(runner_obj);
  auto& runner = runner_obj.cast<dtfs::runtime::StepRunner&>();
  std::vector<int64_t> rows;
  std::vector<std::vector<dtfs::runtime::LoopSlot>> slots;
  for (auto item : buckets) {
    py::tuple t = item.cast<py::tuple>();
    TORCH_CHECK(t.size() == 2, "bucket entries are (rows, slots)");
    rows.push_back(t[0].cast<int64_t>());
    std::vector<dtfs::runtime::LoopSlot> v;
    for (auto d : t[1].cast<py::list>()) v.push_back(loop_slot_from(d.cast<py::dict>(), &p->keep));
    slots.push_back(std::move(v));
  }
  auto ar = dtfs_live::arenas_from(arenas, true, &p->keep);
  p->backend = std::make_unique<GpuBackend>(&runner, std::move(rows), std::move(slots));
  if (auto* sc = dtfs_live::scatter_from(scatter, &p->keep)) {
    const auto lc = dtfs_live::live_config_from(cfg);
    p->backend->set_scatter(sc, share_rows.cast<std::vector<int64_t>>(), lc.step_timeout_us);
  }
  p->srv = std::make_unique<dtfs::runtime::LiveServer>(p->backend.get(), dtfs_live::live_config_from(cfg),
                                                       std::move(ar), ctl);
  return p;
}

}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "distributed_tf_serving_amd gfx950 kernels (MFMA GEMM, embedding gather/bag, interactions, sort)";
  m.def("pack_ids", &pack_ids, py::arg("ids"), py::arg("modulo") = 0, py::arg("modulo_f") = py::none(),
        py::arg("offset_f") = py::none());
  m.def("embed", &embed, py::arg("table"), py::arg("lin"), py::arg("ids"), py::arg("wts"), py::arg("modulo"),
        py::arg("modulo_f") = py::none(), py::arg("offset_f") = py::none(), py::arg("bias") = 0.0,
        py::arg("want_x") = true, py::arg("want_fm") = false, py::arg("fm2") = false, py::arg("out_x") = py::none(),
        py::arg("validate_tables") = false, py::arg("shard_lo_f") = py::none(), py::arg("shard_n_f") = py::none(),
        py::arg("k_pad") = 0, py::arg("cross_w") = py::none(), py::arg("cross_c") = py::none());
  m.def("dense_pad", &dense_pad, py::arg("x"), py::arg("n"), py::arg("K"));
  m.def("embed_gemm", &embed_gemm, py::arg("table"), py::arg("lin"), py::arg("arena"), py::arg("ids"), py::arg("wts"),
        py::arg("B"), py::arg("F"), py::arg("modulo"), py::arg("bias"), py::arg("W"), py::arg("b"), py::arg("act"),
        py::arg("fm2"), py::arg("cross_w") = py::none(), py::arg("cross_c") = py::none(),
        py::arg("resolved") = py::none(), py::arg("Wp") = py::none());
  m.def("embed_gemm_resolve", &embed_gemm_resolve, py::arg("table"), py::arg("lin"), py::arg("arena"), py::arg("ids"),
        py::arg("wts"), py::arg("B"), py::arg("F"), py::arg("modulo"), py::arg("bias"), py::arg("n_parts"),
        "gather-GEMM front half (K1 resolve) -> (rows_t, wts_t, parts) for embed_gemm(resolved=...)");
  m.def("embed_arena", &embed_arena, py::arg("table"), py::arg("lin"), py::arg("arena"), py::arg("B"), py::arg("F"),
        py::arg("modulo"), py::arg("bias") = 0.0, py::arg("want_x") = true, py::arg("want_fm") = false,
        py::arg("fm2") = false, py::arg("out_x") = py::none(), py::arg("k_pad") = 0, py::arg("cross_w") = py::none(),
        py::arg("cross_c") = py::none());
  m.def("embedding_bag", &embedding_bag, py::arg("table"), py::arg("indices"), py::arg("offsets"),
        py::arg("per_sample_weights") = py::none(), py::arg("modulo") = 0, py::arg("mean") = false,
        py::arg("out_bf16") = false, py::arg("out") = py::none());
  m.def("gemm", &gemm, py::arg("A"), py::arg("W"), py::arg("bias") = py::none(), py::arg("epi") = 0,
        py::arg("x0") = py::none(), py::arg("xl") = py::none(), py::arg("out_f32") = false,
        py::arg("sa") = py::none(), py::arg("sw") = py::none(), py::arg("out") = py::none(),
        py::arg("variant") = 0, py::arg("sa_blk") = py::none(), py::arg("q_out") = py::none(),
        py::arg("sq_out") = py::none());
  m.def("cross_v1", &cross_v1, py::arg("x0"), py::arg("w"), py::arg("b"), py::arg("want_x") = true,
        py::arg("head_w") = py::none());
  m.def("dot_interaction", &dot_interaction, py::arg("dense"), py::arg("emb"), py::arg("out_cols") = 0,
        py::arg("emb_off") = py::none(), py::arg("emb_stride") = py::none());
  m.def("shard_route", &shard_route, py::arg("ids"), py::arg("arena"), py::arg("B"), py::arg("F"), py::arg("W"),
        py::arg("tm"), py::arg("col"), py::arg("mod"), py::arg("off"), py::arg("out") = py::none(),
        py::arg("hot") = 1, py::arg("wts") = py::none(), py::arg("out_w") = py::none(),
        "K1b routing: rows (+ weights) of every candidate's owned-table ids grouped by owner rank");
  m.def("dot_interaction_gather_peer", &dot_interaction_gather_peer, py::arg("dense"), py::arg("ids"),
        py::arg("arena"), py::arg("id_col0"), py::arg("cbase"), py::arg("towner"), py::arg("toff"), py::arg("trows"),
        py::arg("tremote"), py::arg("chunk_shift"), py::arg("cache") = py::none(), py::arg("stats") = py::none(),
        py::arg("ring") = py::none(), py::arg("ring_ctr") = py::none(), py::arg("sample_every") = 0,
        py::arg("out_cols") = 0,
        "K1 + K5 with the rows read where they live (peer stores over xGMI, replica cache first)");
  m.def("peer_bag", &peer_bag, py::arg("ids"), py::arg("wts"), py::arg("arena"), py::arg("B"), py::arg("col0"),
        py::arg("hot"), py::arg("cbase"), py::arg("towner"), py::arg("toff"), py::arg("trows"), py::arg("tremote"),
        py::arg("chunk_shift"), py::arg("cache") = py::none(), py::arg("stats") = py::none(),
        py::arg("ring") = py::none(), py::arg("ring_ctr") = py::none(), py::arg("sample_every") = 0, py::arg("out"),
        "K1b multi-hot bags with the rows read where they live -> bf16 [B, T, 64]");
  m.def("peer_cache_fill", &peer_cache_fill, py::arg("keys"), py::arg("slots"), py::arg("cbase"), py::arg("towner"),
        py::arg("toff"), py::arg("trows"), py::arg("tremote"), py::arg("chunk_shift"), py::arg("rows"),
        "replica cache: copy the keys' table rows into their slots");
  m.def("device_alloc", &device_alloc, py::arg("nbytes"), py::arg("like"),
        "uint8 device buffer of exactly nbytes (its own hipMalloc allocation)");
  m.def("cache_index_build", &cache_index_build, py::arg("keys"), py::arg("slots"), py::arg("entries"),
        "replica cache: open-addressing index keys -> slots ({key, slot} entries pre-filled with -1)");
  m.def("ipc_export", &ipc_export, py::arg("t"), "(IPC handle bytes, byte offset) of a device tensor's allocation");
  m.def("ipc_open", &ipc_open, py::arg("handle"), py::arg("offset"), py::arg("shape"), py::arg("like"),
        "map a peer's ipc_export as a tensor (dtype / device of `like`)");
  m.def("head", &head, py::arg("x"), py::arg("w"), py::arg("bias") = 0.0, py::arg("extra") = py::none(),
        py::arg("sigmoid") = true);
  m.def("gemm_head", &gemm_head, py::arg("A"), py::arg("W"), py::arg("bias"), py::arg("act"), py::arg("hw"),
        py::arg("hbias") = 0.0, py::arg("extra") = py::none(), py::arg("sigmoid") = true, py::arg("out") = py::none());
  m.def("mlp_tail", &mlp_tail, py::arg("X"), py::arg("W2p"), py::arg("b2"), py::arg("act2"), py::arg("W3p"),
        py::arg("b3"), py::arg("act3"), py::arg("hw"), py::arg("hbias") = 0.0, py::arg("extra") = py::none(),
        py::arg("sigmoid") = true, py::arg("out") = py::none());
  m.def("gather_mlp", &gather_mlp, py::arg("table"), py::arg("lin"), py::arg("arena"), py::arg("ids"),
        py::arg("wts"), py::arg("B"), py::arg("F"), py::arg("modulo"), py::arg("bias"), py::arg("W1p"), py::arg("b1"),
        py::arg("W2p"), py::arg("b2"), py::arg("act2"), py::arg("W3p"), py::arg("b3"), py::arg("act3"), py::arg("hw"),
        py::arg("hbias"), py::arg("fm"), py::arg("sigmoid") = true, py::arg("out") = py::none(),
        "DeepFM / Wide&Deep tower in one launch: resolve + gather + FM + 3 MLP layers + head (gather_mlp.hip)");
  m.def("set_embed_wave_cap", &dtfs::set_embed_wave_cap, py::arg("waves"), py::arg("rows_in_flight") = 1,
        "pipelined embedding gather geometry: resident-wave cap (0 = one row per wave) and rows in flight per "
        "wave (1 or 2); tuning sweeps and tests");
  m.def("quant_rows_fp8", &quant_rows_fp8, py::arg("x"), py::arg("k_pad") = 1);
  m.def("dot_interaction_gather", &dot_interaction_gather, py::arg("dense"), py::arg("table"), py::arg("ids"),
        py::arg("modulo_f"), py::arg("offset_f"), py::arg("out_cols") = 0);
  m.def("bottom_mlp3", &bottom_mlp3, py::arg("wts"), py::arg("nd"), py::arg("W1"), py::arg("b1"), py::arg("W2"),
        py::arg("b2"), py::arg("W3"), py::arg("b3"));
  m.def("bottom_mlp3_arena", &bottom_mlp3_arena, py::arg("arena"), py::arg("B"), py::arg("nd"), py::arg("W1"),
        py::arg("b1"), py::arg("W2"), py::arg("b2"), py::arg("W3"), py::arg("b3"));
  m.def("dot_interaction_gather_arena", &dot_interaction_gather_arena, py::arg("dense"), py::arg("table"),
        py::arg("arena"), py::arg("id_col0"), py::arg("modulo_f"), py::arg("offset_f"), py::arg("out_cols") = 0);
  m.def("cross_gemm_fp8", &cross_gemm_fp8, py::arg("q"), py::arg("sx"), py::arg("Wq"), py::arg("sw"), py::arg("bias"),
        py::arg("x0"), py::arg("xl"), py::arg("want_z") = true, py::arg("head_w") = py::none());
  m.def("cross_combine", &cross_combine, py::arg("y"), py::arg("x0"), py::arg("xl"), py::arg("want_z") = true,
        py::arg("k_pad") = 0, py::arg("head_w") = py::none(),
        "split DCN-v2 cross layer: z = x0*y + xl, optionally quantised (e4m3 + row scale) and/or dotted with head_w");
  m.def("unpack_arena", &unpack_arena, py::arg("arena"), py::arg("packed"), py::arg("fields"),
        py::arg("narrow_modulo") = 0);
  m.def("arena_varint_decode", &arena_varint_decode, py::arg("arena"), py::arg("blocks") = 256);
  m.def("pull_host", &pull_host, py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("blocks") = 128);
  // stream-ordered 32-bit flag write / wait (a lighter cross-queue dependency
  // than an event; tools/studies/step_gap_study.py)
  m.def(
      "stream_write_u32",
      [](uintptr_t stream, torch::Tensor flag, uint32_t value) {
        TORCH_CHECK(flag.is_cuda() && flag.scalar_type() == torch::kInt32 && flag.numel() >= 1, "flag: int32 GPU tensor");
        check_hip(hipStreamWriteValue32(reinterpret_cast<hipStream_t>(stream), flag.data_ptr(), value, 0),
                  "hipStreamWriteValue32");
      },
      py::arg("stream"), py::arg("flag"), py::arg("value"));
  m.def(
      "stream_wait_u32",
      [](uintptr_t stream, torch::Tensor flag, uint32_t value) {
        TORCH_CHECK(flag.is_cuda() && flag.scalar_type() == torch::kInt32 && flag.numel() >= 1, "flag: int32 GPU tensor");
        check_hip(hipStreamWaitValue32(reinterpret_cast<hipStream_t>(stream), flag.data_ptr(), value,
                                       hipStreamWaitValueGte, 0xffffffffu),
                  "hipStreamWaitValue32");
      },
      py::arg("stream"), py::arg("flag"), py::arg("value"));
  m.def("sort_scores", &sort_scores, py::arg("scores"), py::arg("descending") = false, py::arg("k") = -1);
  m.def("sort_max_elems", &dtfs::sort_max_elems);

  py::class_<dtfs::runtime::StepRunner>(m, "StepRunner",
                                        "Native per-GPU step launcher: SDMA H2D + graph launch per pipeline slot")
      .def(py::init<int, int>(), py::arg("device"), py::arg("slots"))
      .def_property_readonly("aux_cus", &dtfs::runtime::StepRunner::aux_cus)
      .def(
          "launch",
          [](dtfs::runtime::StepRunner& r, int slot, torch::Tensor dst, torch::Tensor src, int64_t nbytes,
             uintptr_t graph_exec) {
            TORCH_CHECK(dst.is_cuda() && dst.is_contiguous(), "dst must be a contiguous GPU tensor");
            TORCH_CHECK(src.device().is_cpu() && src.is_contiguous() && src.is_pinned(),
                        "src must be a contiguous pinned host tensor");
            TORCH_CHECK(nbytes >= 0 && nbytes <= int64_t(dst.nbytes()) && nbytes <= int64_t(src.nbytes()),
                        "nbytes out of range");
            TORCH_CHECK(graph_exec != 0, "null graph exec");
            r.launch(slot, dst.data_ptr(), src.data_ptr(), nbytes, reinterpret_cast<hipGraphExec_t>(graph_exec));
          },
          py::arg("slot"), py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("graph_exec"))
      .def(
          "launch_fanout",
          [](dtfs::runtime::StepRunner& r, int slot, torch::Tensor h2d_dst, torch::Tensor h2d_src, int64_t h2d_bytes,
             uintptr_t ingress_exec, dtfs::comm::RcclComm& cin, int mode, torch::Tensor send, torch::Tensor recv,
             uintptr_t forward_exec, dtfs::comm::RcclComm& cout, torch::Tensor scores, torch::Tensor back,
             torch::Tensor h_out, int64_t d2h_bytes, uintptr_t resolve_exec) {
            TORCH_CHECK(h2d_src.device().is_cpu() && h2d_src.is_pinned(), "h2d_src must be pinned host memory");
            TORCH_CHECK(h2d_bytes >= 0 && h2d_bytes <= int64_t(h2d_dst.nbytes()) &&
                            h2d_bytes <= int64_t(h2d_src.nbytes()),
                        "h2d_bytes out of range");
            auto s = make_fanout_step(h2d_dst, ingress_exec, cin, mode, send, recv, forward_exec, cout, scores, back,
                                      h_out, d2h_bytes);
            s.h2d_src = h2d_src.data_ptr();
            s.h2d_bytes = h2d_bytes;
            s.resolve = reinterpret_cast<hipGraphExec_t>(resolve_exec);
            r.launch_fanout(slot, s);
          },
          py::arg("slot"), py::arg("h2d_dst"), py::arg("h2d_src"), py::arg("h2d_bytes"), py::arg("ingress_exec"),
          py::arg("cin"), py::arg("mode"), py::arg("send"), py::arg("recv"), py::arg("forward_exec"), py::arg("cout"),
          py::arg("scores"), py::arg("back"), py::arg("h_out"), py::arg("d2h_bytes"), py::arg("resolve_exec") = 0)
      .def(
          "launch_program",
          [](dtfs::runtime::StepRunner& r, int slot, py::dict program, torch::Tensor h2d_src, int64_t h2d_bytes) {
            std::vector<py::object> keep;  // the caller keeps the program's objects alive while it runs
            auto p = program_from(program, &keep);
            torch::Tensor dst = program["h2d_dst"].cast<torch::Tensor>();
            TORCH_CHECK(h2d_src.device().is_cpu() && h2d_src.is_pinned(), "h2d_src must be pinned host memory");
            TORCH_CHECK(h2d_bytes >= 0 && h2d_bytes <= int64_t(dst.nbytes()) && h2d_bytes <= int64_t(h2d_src.nbytes()),
                        "h2d_bytes out of range");
            r.launch_program(slot, p, h2d_src.data_ptr(), h2d_bytes);
          },
          py::arg("slot"), py::arg("program"), py::arg("h2d_src"), py::arg("h2d_bytes"))
      .def("wait", &dtfs::runtime::StepRunner::wait, py::arg("slot"), py::call_guard<py::gil_scoped_release>())
      .def(
          "wait_for",
          [](dtfs::runtime::StepRunner& r, int slot, double timeout_s, std::vector<dtfs::comm::RcclComm*> comms) {
            std::string err;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = r.wait_for(slot, int64_t(timeout_s * 1e6), comms, &err);
            }
            return py::make_tuple(ok, err);
          },
          py::arg("slot"), py::arg("timeout_s"), py::arg("comms") = std::vector<dtfs::comm::RcclComm*>(),
          "Bounded wait for the slot's step: (ok, error). Also polls the communicators' async errors.")
      .def("query", &dtfs::runtime::StepRunner::query, py::arg("slot"))
      .def_property_readonly("slots", &dtfs::runtime::StepRunner::slots)
      .def_property("feed_h2d", &dtfs::runtime::StepRunner::feed_h2d, &dtfs::runtime::StepRunner::set_feed_h2d,
                    "local steps: a feeder thread enqueues each step's kernels once the host sees its H2D landed "
                    "(True, default) instead of a device-side wait on the copy's event")
      .def_property("host_wait_h2d", &dtfs::runtime::StepRunner::host_wait_h2d,
                    &dtfs::runtime::StepRunner::set_host_wait_h2d,
                    "local steps: wait for each step's H2D on the host (True) or on the device (False)")
      .def_property_readonly("compute_stream",
                             [](const dtfs::runtime::StepRunner& r) { return reinterpret_cast<uintptr_t>(r.compute_stream()); });

  py::class_<dtfs::runtime::KernelSequence>(m, "KernelSequence",
                                            "A captured HIP graph replayed as direct kernel launches")
      .def(py::init([](uintptr_t graph) {
             TORCH_CHECK(graph != 0, "null hipGraph_t (capture with torch.cuda.CUDAGraph(keep_graph=True))");
             return std::make_unique<dtfs::runtime::KernelSequence>(reinterpret_cast<hipGraph_t>(graph));
           }),
           py::arg("graph"))
      .def(
          "launch",
          [](const dtfs::runtime::KernelSequence& s, uintptr_t stream) {
            s.launch(stream ? reinterpret_cast<hipStream_t>(stream)
                            : c10::hip::getCurrentHIPStream().stream());
          },
          py::arg("stream") = 0)
      .def_property_readonly("size", &dtfs::runtime::KernelSequence::size)
      .def("describe", &dtfs::runtime::KernelSequence::describe);

  {
    py::class_<PyGpuLive> c(m, "LiveServer",
                            "Live serving core (csrc/runtime/live_server.h) on this GPU: requests are batched into "
                            "pinned arenas and run as captured step kernels (or the fan-out step)");
    c.def(py::init(&make_gpu_live), py::arg("runner"), py::arg("config"), py::arg("buckets"), py::arg("arenas"),
          py::arg("control") = py::none(), py::arg("scatter") = py::none(), py::arg("share_rows") = py::none());
    dtfs_live::def_live_methods(c);
  }
  dtfs_live::def_step_control(m);
  dtfs_live::def_grpc_front<PyGpuLive>(m);
  {
    auto sc = dtfs_live::def_shared_scatter(m);
    sc.def(
          "register_with_gpu",
          [](dtfs::runtime::SharedScatter& s) {
            // every rank pins the whole mapping for its own GPU: its DMA reads
            // rank 0's arenas, its head kernel writes the shared scores
            check_hip(hipHostRegister(s.base(), s.bytes(), hipHostRegisterMapped), "hipHostRegister(shared scatter)");
            s.set_on_unmap([](void* p, size_t) { (void)hipHostUnregister(p); });
          })
        .def(
            "launch",
            [](dtfs::runtime::SharedScatter& s, dtfs::runtime::StepRunner& r, int slot, int64_t rows_per_rank,
               c10::optional<torch::Tensor> arena, torch::Tensor dst, py::object seq, uintptr_t graph_exec,
               double timeout_s) {
              TORCH_CHECK(dst.is_cuda() && dst.is_contiguous() && dst.numel() >= s.arena_cap(),
                          "dst must be a device arena of the segment's capacity");
              const dtfs::runtime::KernelSequence* ks =
                  seq.is_none() ? nullptr : &seq.cast<dtfs::runtime::KernelSequence&>();
              TORCH_CHECK(ks || graph_exec, "need a kernel sequence or a graph");
              const uint8_t* a = arena ? static_cast<const uint8_t*>(arena->data_ptr()) : nullptr;
              return scatter_step(r, s, slot, rows_per_rank, a, dst.data_ptr(), int64_t(dst.nbytes()), ks,
                                  reinterpret_cast<hipGraphExec_t>(graph_exec), int64_t(timeout_s * 1e6));
            },
            py::arg("runner"), py::arg("slot"), py::arg("rows_per_rank"), py::arg("arena"), py::arg("dst"),
            py::arg("seq"), py::arg("graph_exec"), py::arg("timeout_s") = 10.0,
            "engine-level shared-scatter step (self-check); returns the step index")
        .def(
            "wait",
            [](dtfs::runtime::SharedScatter& s, dtfs::runtime::StepRunner& r, int slot, uint64_t k, double timeout_s) {
              std::string err;
              bool ok;
              {
                py::gil_scoped_release nogil;
                ok = scatter_wait(r, s, slot, k, int64_t(timeout_s * 1e6), {}, &err);
              }
              return py::make_tuple(ok, err);
            },
            py::arg("runner"), py::arg("slot"), py::arg("step"), py::arg("timeout_s") = 10.0);
  }

  m.def("rccl_set_library", &dtfs::comm::set_library, py::arg("path"));
  // NUMA-local pinned host memory (runtime/numa.h): pages placed on `node`
  // first, then registered with the GPU; freed by unregister + munmap
  m.def(
      "alloc_pinned_on_node",
      [](int64_t bytes, int node) {
        void* p = dtfs::runtime::alloc_on_node(size_t(bytes), node);
        if (hipHostRegister(p, size_t(bytes), hipHostRegisterDefault) != hipSuccess) {
          dtfs::runtime::free_on_node(p, size_t(bytes));
          throw std::runtime_error("hipHostRegister failed");
        }
        const size_t n = size_t(bytes);
        return torch::from_blob(p, {bytes},
                                [n](void* q) {
                                  (void)hipHostUnregister(q);
                                  dtfs::runtime::free_on_node(q, n);
                                },
                                torch::TensorOptions().dtype(torch::kUInt8));
      },
      py::arg("bytes"), py::arg("node"));
  m.def(
      "pci_bus_id",
      [](int device) {
        char buf[64] = {0};
        if (hipDeviceGetPCIBusId(buf, sizeof(buf), device) != hipSuccess) return std::string();
        return std::string(buf);
      },
      py::arg("device"), "PCI bus id of a GPU (\"0000:65:00.0\"), for its NUMA node");
  m.def("rccl_unique_id", []() { return py::bytes(dtfs::comm::unique_id()); });
  py::class_<dtfs::comm::RcclComm>(m, "RcclComm", "Native RCCL communicator (fan-out collectives over xGMI)")
      .def(py::init([](py::bytes uid, int nranks, int rank, int device) {
             std::string id(uid);  // convert while holding the GIL
             py::gil_scoped_release nogil;  // ncclCommInitRank blocks until every rank joins
             return std::make_unique<dtfs::comm::RcclComm>(id, nranks, rank, device);
           }),
           py::arg("uid"), py::arg("nranks"), py::arg("rank"), py::arg("device"))
      .def_property_readonly("rank", &dtfs::comm::RcclComm::rank)
      .def_property_readonly("nranks", &dtfs::comm::RcclComm::nranks)
      .def(
          "alltoall",
          [](dtfs::comm::RcclComm& c, torch::Tensor send, torch::Tensor recv) {
            TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                        "contiguous GPU tensors");
            TORCH_CHECK(send.nbytes() == recv.nbytes() && send.nbytes() % c.nranks() == 0,
                        "send/recv must be equal and divisible by the world size");
            c10::DeviceGuard g(send.device());
            c.alltoall(send.data_ptr(), recv.data_ptr(), send.nbytes() / c.nranks(), cur_stream(send));
          },
          py::arg("send"), py::arg("recv"))
      .def(
          "allgather",
          [](dtfs::comm::RcclComm& c, torch::Tensor send, torch::Tensor recv) {
            TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                        "contiguous GPU tensors");
            TORCH_CHECK(recv.nbytes() == send.nbytes() * c.nranks(), "recv must be world x send");
            c10::DeviceGuard g(send.device());
            c.allgather(send.data_ptr(), recv.data_ptr(), send.nbytes(), cur_stream(send));
          },
          py::arg("send"), py::arg("recv"))
      .def(
          "gather",
          [](dtfs::comm::RcclComm& c, torch::Tensor send, torch::Tensor recv, int root) {
            TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                        "contiguous GPU tensors");
            TORCH_CHECK(root >= 0 && root < c.nranks(), "bad root");
            TORCH_CHECK(c.rank() != root || recv.nbytes() == send.nbytes() * c.nranks(), "root recv must be world x send");
            c10::DeviceGuard g(send.device());
            c.gather(send.data_ptr(), recv.data_ptr(), send.nbytes(), root, cur_stream(send));
          },
          py::arg("send"), py::arg("recv"), py::arg("root") = 0)
      .def(
          "scatter",
          [](dtfs::comm::RcclComm& c, torch::Tensor send, torch::Tensor recv, int root) {
            TORCH_CHECK(send.is_cuda() && recv.is_cuda() && send.is_contiguous() && recv.is_contiguous(),
                        "contiguous GPU tensors");
            TORCH_CHECK(root >= 0 && root < c.nranks(), "bad root");
            TORCH_CHECK(c.rank() != root || send.nbytes() == recv.nbytes() * c.nranks(), "root send must be world x recv");
            c10::DeviceGuard g(recv.device());
            c.scatter(send.data_ptr(), recv.data_ptr(), recv.nbytes(), root, cur_stream(recv));
          },
          py::arg("send"), py::arg("recv"), py::arg("root") = 0)
      .def(
          "peer_prepare", [](dtfs::comm::RcclComm& c, uint64_t cap) { return py::bytes(c.peer_prepare(cap)); },
          py::arg("cap"),
          "Allocate and export this rank's one-shot exchange mailbox (collective setup, step 1); returns its IPC handle")
      .def(
          "peer_enable",
          [](dtfs::comm::RcclComm& c, std::vector<py::bytes> handles, double timeout_s) {
            std::vector<std::string> h;
            for (auto& b : handles) h.emplace_back(std::string(b));
            c.peer_enable(h, timeout_s);
          },
          py::arg("handles"), py::arg("timeout_s") = 5.0,
          "Map every rank's mailbox (handles in rank order); messages <= cap then bypass RCCL")
      .def("can_access_device", &dtfs::comm::RcclComm::can_access_device, py::arg("device"),
           "hipDeviceCanAccessPeer from this communicator's device")
      .def_property_readonly("peer_enabled", &dtfs::comm::RcclComm::peer_enabled)
      .def_property_readonly("peer_cap", &dtfs::comm::RcclComm::peer_cap)
      .def_property_readonly("peer_exchanges", &dtfs::comm::RcclComm::peer_exchanges)
      .def("async_error", &dtfs::comm::RcclComm::async_error)
      .def("abort", &dtfs::comm::RcclComm::abort)
      .def_property_readonly("aborted", &dtfs::comm::RcclComm::aborted);
}

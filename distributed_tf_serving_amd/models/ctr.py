"""CTR model families served by a shard backend.

The reference serves a SavedModel called "DCN" whose inputs are
``feat_ids`` int64 [B, F] and ``feat_wts`` float [B, F] and whose output
``prediction_node`` is one CTR per candidate (reference DCNClient.java:33-35,
97-108, 162). The graph itself is external (TF-Serving); SURVEY.md §2.2 E4
lists the implied compute. Every family below consumes exactly that input
signature (libsvm-style: an id and a weight per field; for DLRM the leading
``num_dense`` fields carry dense values in ``feat_wts``) and produces
sigmoid CTR scores, so any of them can stand behind the reference client.

Forward passes are built only from :mod:`distributed_tf_serving_amd.ops`, so
GPU tensors run the gfx950 kernels and CPU tensors run the fp32 reference
math. Weights are random-init from ``cfg.seed`` (no checkpoints exist).

===========  ==========================================================
family       forward
===========  ==========================================================
wdl          sigmoid(wide(ids, wts) + head(MLP(emb)))
deepfm       sigmoid(FM1 + FM2 + head(MLP(emb)))
dcn          sigmoid(w_c . cross_v1^L(emb) + head(MLP(emb)))
dcn_v2       sigmoid(w_c . cross_v2^L(emb) + head(MLP(emb)))  (fp8 towers opt.)
dlrm         sigmoid(head(topMLP(dot(botMLP(dense), emb_t))))
===========  ==========================================================
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
from torch import nn

from .. import ops
from ..config import ModelConfig
from .layers import DTYPES, MLP, Dense, hashed_uniform_rows_, init_uniform_, make_generator, pad8


class CTRModel(nn.Module):
    """Base: holds config, exposes ``forward(ids, wts) -> CTR [B] fp32``."""

    family = "base"
    # DeepFM / WDL: run the first MLP layer as the gather-GEMM where it applies
    # (_gather_gemm); tests switch it off per instance to compare the two paths
    use_gather_gemm = True

    def __init__(self, cfg: ModelConfig, device="cpu"):
        super().__init__()
        self.cfg = cfg
        self.device_ = torch.device(device)
        self.dtype = DTYPES[cfg.param_dtype]
        self.gen = make_generator(cfg.seed, self.device_)

    # -- metadata ----------------------------------------------------------
    def signature(self) -> Dict[str, Dict]:
        F = self.cfg.num_fields
        return {
            "inputs": {"feat_ids": ("DT_INT64", [-1, F]), "feat_wts": ("DT_FLOAT", [-1, F])},
            # ranked outputs: produced when named in output_filter (serving/service.py)
            "outputs": {"prediction_node": ("DT_FLOAT", [-1]), "sorted_prediction": ("DT_FLOAT", [-1]),
                        "sorted_index": ("DT_INT64", [-1])},
            "method_name": "tensorflow/serving/predict",
        }

    def param_bytes(self) -> int:
        n = sum(p.numel() * p.element_size() for p in self.parameters())
        n += sum(b.numel() * b.element_size() for b in self.buffers())
        return n

    def _embedding_table(self, rows: int, dim: int) -> nn.Parameter:
        t = torch.empty(rows, dim, dtype=self.dtype, device=self.device_)
        init_uniform_(t, 1.0 / math.sqrt(dim), self.gen)
        return nn.Parameter(t, requires_grad=False)

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, wts: Optional[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """CTR [B] fp32. ``out`` (fp32 [B], device or pinned host) receives the
        scores straight from the head kernel (no separate D2H copy)."""
        # bf16 weights go to the gather as they are (narrow fan-out rows carry fp32)
        if wts is not None and wts.dtype not in (torch.float32, torch.bfloat16):
            wts = wts.float()
        return self._forward(ids, wts, out)

    def _forward(self, ids, wts, out=None, resolved=None):  # pragma: no cover - abstract
        raise NotImplementedError

    # families whose only use of ids / weights is the first embedding gather
    # can read them straight from a request arena (ops.ArenaRows)
    supports_arena = False

    def _gather_gemm(self, ids, wts, fm2: bool) -> bool:
        """The first MLP layer runs as the gather-GEMM (ops.embed_gemm): GPU,
        bf16 towers of >= 2 layers, a shape the kernel covers."""
        layers = self.mlp.layers
        first = layers[0]
        on_gpu = ids.arena.is_cuda if isinstance(ids, ops.ArenaRows) else ids.is_cuda
        return (on_gpu and self.use_gather_gemm and len(layers) >= 2 and not first.fp8
                and (wts is None or wts.dtype == torch.float32)
                and first.act in ("relu", "none") and first.k == first.in_dim
                and ops.embed_gemm_ok(self.emb, first.weight, int(ids.shape[0]), fm2))

    def _gather_mlp(self, ids, wts, fm2: bool) -> bool:
        """The whole tower runs as ONE kernel (ops.gather_mlp: gather + FM + the
        three MLP layers + head, h1 / h2 in LDS): the gather-GEMM applies and
        the tower is 64F -> 1024 -> 512 -> 256 on a batch that fills the GPU."""
        return (self.use_gather_mlp and self._gather_gemm(ids, wts, fm2)
                and ops.gather_mlp_ok(self.emb, self.mlp.layers, int(ids.shape[0])))

    # module-level A/B switch for studies (tools/studies): False keeps the
    # two-kernel form (gather-GEMM + MLP tail)
    use_gather_mlp = True

    def _resolve_applies(self, ids, wts) -> bool:
        """The step runs the gather-GEMM (so its resolve pass can move to the aux lane)."""
        return False

    def _resolve(self, ids, wts):
        """The gather-GEMM's front half of this family (ops.embed_gemm_resolve)."""
        raise NotImplementedError

    # A local GPU step as a two-lane program (parallel/step_program.py): the
    # gather-GEMM's resolve pass of step k+1 runs on the aux lane right after
    # its H2D, while the compute lane finishes step k (DTFS_RESOLVE_LANE=1;
    # off by default since the one-wave gather-GEMM leaves it no registers to
    # co-run in, parallel/fanout.py _program_enabled).
    resolve_lane = False

    def build_program(self, ids, wts, B: int, bufs: dict, out: Optional[torch.Tensor] = None,
                      state: Optional[dict] = None) -> list:
        from ..parallel import step_program as sp

        st = {} if state is None else state
        if self.resolve_lane and self._resolve_applies(ids, wts):
            # (gating step k+1's resolve on step k's tower - so it runs beside the
            # head instead of GEMM2 - measured no better: 105.4 vs 106.1 / 104.0 M
            # serial on one box, profiles/r04_session2.md; round 5, gated behind
            # the one-wave gather-GEMM to run beside the fused MLP tail: 107.9 /
            # 112.8 vs 126.1 / 126.1 M one-stream, interleaved on one box)
            def resolve():
                st["resolved"] = self._resolve(ids, wts)

            def main():
                st["scores"] = self._forward(ids, wts, out, resolved=st["resolved"])

            return [sp.Kernels(sp.AUX, resolve, "resolve"), sp.Sync("record", sp.AUX, 0),
                    sp.Sync("wait", sp.COMPUTE, 0), sp.Kernels(sp.COMPUTE, main, "forward")]

        def fwd():
            st["scores"] = self._forward(ids, wts, out)

        return [sp.Sync("record", sp.AUX, 0), sp.Sync("wait", sp.COMPUTE, 0), sp.Kernels(sp.COMPUTE, fwd, "forward")]

    @torch.no_grad()
    def forward_arena(self, arena: torch.Tensor, B: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """CTR [B] for the first B candidate rows of a (device) request arena."""
        if not self.supports_arena:
            raise NotImplementedError(f"{self.family} reads dense features; unpack the arena first")
        return self._forward(ops.ArenaRows(arena, int(B), self.cfg.num_fields), None, out)


class WideDeep(CTRModel):
    family = "wdl"
    supports_arena = True

    def __init__(self, cfg: ModelConfig, device="cpu"):
        super().__init__(cfg, device)
        V, D, F = cfg.vocab_size, cfg.embed_dim, cfg.num_fields
        self.emb = self._embedding_table(V, D)
        self.wide = nn.Parameter(init_uniform_(torch.empty(V, device=self.device_), 0.05, self.gen), requires_grad=False)
        self.wide_bias = 0.0
        self.mlp = MLP(F * D, cfg.mlp_dims, self.dtype, self.device_, self.gen)
        self.head_w = nn.Parameter(init_uniform_(torch.empty(self.mlp.out_dim, device=self.device_), 0.05, self.gen),
                                   requires_grad=False)
        self.head_b = 0.0

    def _front(self, ids, wts):
        return ops.embed(self.emb, ids, wts, lin=self.wide, modulo=self.cfg.vocab_size, bias=self.wide_bias,
                         want_x=True, want_fm=True, fm2=False)

    resolve_lane = True

    def _resolve_applies(self, ids, wts) -> bool:
        # the one-launch tower resolves its rows itself: no separate pass to move
        return self._gather_gemm(ids, wts, fm2=False) and not self._gather_mlp(ids, wts, fm2=False)

    def _resolve(self, ids, wts):
        return ops.embed_gemm_resolve(self.emb, ids, wts, self.wide, self.cfg.vocab_size, self.wide_bias, False)

    def _gg_front(self, ids, wts, resolved=None):
        first = self.mlp.layers[0]
        h, wide = ops.embed_gemm(self.emb, ids, wts, self.wide, self.cfg.vocab_size, self.wide_bias, first.weight,
                                 first.bias, first.act, fm2=False, resolved=resolved,
                                 packed_w=lambda: first.packed("32"))
        return h, wide, self.head_w, self.head_b

    def _forward(self, ids, wts, out=None, resolved=None):
        if self._gather_mlp(ids, wts, fm2=False):  # the whole tower in one launch
            return ops.gather_mlp(self.emb, ids, wts, self.wide, self.cfg.vocab_size, self.wide_bias, self.mlp.layers,
                                  self.head_w, self.head_b, fm=False, out=out)
        if self._gather_gemm(ids, wts, fm2=False):
            h, wide, hw, hb = self._gg_front(ids, wts, resolved)
            return self.mlp.forward_head(h, hw, hb, extra=wide, out=out, start=1)
        x, wide = self._front(ids, wts)
        return self.mlp.forward_head(x, self.head_w, self.head_b, extra=wide, out=out)


class DeepFM(CTRModel):
    family = "deepfm"
    supports_arena = True

    def __init__(self, cfg: ModelConfig, device="cpu"):
        super().__init__(cfg, device)
        V, D, F = cfg.vocab_size, cfg.embed_dim, cfg.num_fields
        self.emb = self._embedding_table(V, D)
        self.lin = nn.Parameter(init_uniform_(torch.empty(V, device=self.device_), 0.01, self.gen), requires_grad=False)
        self.fm_bias = 0.0
        self.mlp = MLP(F * D, cfg.mlp_dims, self.dtype, self.device_, self.gen, fp8=cfg.gemm_dtype == "fp8")
        self.head_w = nn.Parameter(init_uniform_(torch.empty(self.mlp.out_dim, device=self.device_), 0.05, self.gen),
                                   requires_grad=False)
        self.head_b = 0.0

    def _front(self, ids, wts):
        return ops.embed(self.emb, ids, wts, lin=self.lin, modulo=self.cfg.vocab_size, bias=self.fm_bias,
                         want_x=True, want_fm=True, fm2=True)

    resolve_lane = True

    def _resolve_applies(self, ids, wts) -> bool:
        # the one-launch tower resolves its rows itself: no separate pass to move
        return self._gather_gemm(ids, wts, fm2=True) and not self._gather_mlp(ids, wts, fm2=True)

    def _resolve(self, ids, wts):
        return ops.embed_gemm_resolve(self.emb, ids, wts, self.lin, self.cfg.vocab_size, self.fm_bias, True)

    def _gg_front(self, ids, wts, resolved=None):
        # K1 + K2 inside the first layer's GEMM: x never reaches HBM
        first = self.mlp.layers[0]
        h, fm = ops.embed_gemm(self.emb, ids, wts, self.lin, self.cfg.vocab_size, self.fm_bias, first.weight,
                               first.bias, first.act, fm2=True, resolved=resolved,
                               packed_w=lambda: first.packed("32"))
        return h, fm, self.head_w, self.head_b

    def _forward(self, ids, wts, out=None, resolved=None):
        if self._gather_mlp(ids, wts, fm2=True):  # the whole tower in one launch
            return ops.gather_mlp(self.emb, ids, wts, self.lin, self.cfg.vocab_size, self.fm_bias, self.mlp.layers,
                                  self.head_w, self.head_b, fm=True, out=out)
        if self._gather_gemm(ids, wts, fm2=True):
            h, fm, hw, hb = self._gg_front(ids, wts, resolved)
            return self.mlp.forward_head(h, hw, hb, extra=fm, out=out, start=1)
        x, fm = self._front(ids, wts)
        return self.mlp.forward_head(x, self.head_w, self.head_b, extra=fm, out=out)


class DCN(CTRModel):
    """Deep & Cross Network (v1) - the reference's served model name."""

    family = "dcn"
    supports_arena = True

    def __init__(self, cfg: ModelConfig, device="cpu"):
        super().__init__(cfg, device)
        V, D, F, L = cfg.vocab_size, cfg.embed_dim, cfg.num_fields, cfg.num_cross_layers
        d = F * D
        self.emb = self._embedding_table(V, D)
        self.cross_w = nn.Parameter(init_uniform_(torch.empty(L, d, device=self.device_), 1.0 / math.sqrt(d), self.gen),
                                    requires_grad=False)
        self.cross_b = nn.Parameter(torch.zeros(L, d, device=self.device_), requires_grad=False)
        self.mlp = MLP(d, cfg.mlp_dims, self.dtype, self.device_, self.gen)
        # head over concat(x_L, h): split into the cross part (fused into K3) and the deep part (K6)
        self.head_wc = nn.Parameter(init_uniform_(torch.empty(d, device=self.device_), 0.5 / math.sqrt(d), self.gen),
                                    requires_grad=False)
        self.head_wd = nn.Parameter(init_uniform_(torch.empty(self.mlp.out_dim, device=self.device_), 0.05, self.gen),
                                    requires_grad=False)
        self.head_b = 0.0

    resolve_lane = True

    def _resolve_applies(self, ids, wts) -> bool:
        return self.cfg.num_cross_layers + 1 <= 4 and self._gather_gemm(ids, wts, fm2=True)

    def _resolve(self, ids, wts):
        return ops.embed_gemm_resolve(self.emb, ids, wts, None, self.cfg.vocab_size, 0.0, True)

    def _gg_front(self, ids, wts, resolved=None):
        # gather + cross network + first MLP layer in one kernel (x0 never in HBM)
        first = self.mlp.layers[0]
        h, parts = ops.embed_gemm(self.emb, ids, wts, None, self.cfg.vocab_size, 0.0, first.weight, first.bias,
                                  first.act, fm2=False,
                                  cross=(self.cross_w, self.cross_b, self.head_wc, self._cross_consts()),
                                  resolved=resolved)
        return h, parts, self.head_wd, self.head_b

    def _forward(self, ids, wts, out=None, resolved=None):
        if self.cfg.num_cross_layers + 1 <= 4 and self._gather_gemm(ids, wts, fm2=True):
            h, parts, hw, hb = self._gg_front(ids, wts, resolved)
            return self.mlp.forward_head(h, hw, hb, extra=parts, out=out, start=1)
        # the whole cross network rides on the gather (ops.embed_cross): the
        # wave holding x0 computes its L + 1 weight dot products
        on_gpu = ids.arena.is_cuda if isinstance(ids, ops.ArenaRows) else ids.is_cuda
        x, cross_logit = ops.embed_cross(self.emb, ids, wts, self.cfg.vocab_size, self.cross_w, self.cross_b,
                                         self.head_wc, self._cross_consts() if on_gpu else None)
        return self.mlp.forward_head(x, self.head_wd, self.head_b, extra=cross_logit, out=out)

    def _cross_consts(self):
        """Folded cross weights (ops.cross_v1_consts), recomputed only when the
        weights change (load_state_dict): cached tensors stay valid inside
        captured graphs."""
        key = (self.cross_w._version, self.cross_b._version, self.head_wc._version, self.cross_w.data_ptr())
        if getattr(self, "_cc_key", None) != key:
            rows, c = ops.cross_v1_consts(self.cross_w, self.cross_b, self.head_wc)
            if getattr(self, "_cc", None) is not None and self._cc[0].shape == rows.shape:
                self._cc[0].copy_(rows)  # in place: graphs captured earlier read these buffers
                self._cc[1].copy_(c)
            else:
                self._cc = (rows, c)
            self._cc_key = key
        return self._cc


class DCNv2(CTRModel):
    """DCN-v2: full-rank (or low-rank) matrix cross layers; optional fp8 towers."""

    family = "dcn_v2"
    supports_arena = True

    def __init__(self, cfg: ModelConfig, device="cpu"):
        super().__init__(cfg, device)
        V, D, F, L = cfg.vocab_size, cfg.embed_dim, cfg.num_fields, cfg.num_cross_layers
        d = F * D
        self.d = d
        self.fp8 = cfg.gemm_dtype == "fp8"
        self.emb = self._embedding_table(V, D)
        self.low_rank = cfg.cross_rank > 0
        if self.low_rank:
            r = pad8(cfg.cross_rank)
            self.cross_v = nn.ModuleList([Dense(d, r, "none", self.dtype, self.device_, self.gen, fp8=self.fp8)
                                          for _ in range(L)])
            self.cross_u = nn.ModuleList([Dense(r, d, "none", self.dtype, self.device_, self.gen) for _ in range(L)])
        else:
            self.cross = nn.ModuleList([Dense(d, d, "none", self.dtype, self.device_, self.gen, fp8=self.fp8)
                                        for _ in range(L)])
            for layer in self.cross:  # keep the stacked product well-conditioned
                layer.weight.data.mul_(0.5)
                if self.fp8:
                    layer.quantize_fp8()
        self.mlp = MLP(d, cfg.mlp_dims, self.dtype, self.device_, self.gen, fp8=self.fp8)
        # fp8 towers = the cross layers and the first (2752-deep) MLP layer, 97 % of
        # the FLOPs; the small tail layers stay bf16 so the last layer + head run as
        # one fused kernel writing the scores to pinned memory (fp8 there needs two
        # quant passes, a separate head and a D2H copy: 53 us vs ~37 us per
        # 16384-row step, round 2)
        if self.fp8:
            for layer in self.mlp.layers[1:]:
                layer.fp8 = False
        self.head_wc = nn.Parameter(init_uniform_(torch.empty(d, device=self.device_), 0.5 / math.sqrt(d), self.gen),
                                    requires_grad=False)
        self.head_wd = nn.Parameter(init_uniform_(torch.empty(self.mlp.out_dim, device=self.device_), 0.05, self.gen),
                                    requires_grad=False)
        self.head_b = 0.0

    def _cross_layer(self, i: int, x0: torch.Tensor, xl: torch.Tensor, xq=None):
        """One cross layer with the cross epilogue fused into its GEMM. fp8:
        ``xq`` = (q, row scales) of xl."""
        if self.low_rank:
            # x0 * (U (V xl) + b) + xl : the cross epilogue rides on the U GEMM
            v = self.cross_v[i](xl)
            u = self.cross_u[i]
            return ops.cross_v2(x0, xl, u.weight, u.bias, a=v)
        layer = self.cross[i]
        if self.fp8:
            q, sx = xq if xq is not None else ops.quant_rows_fp8(xl, ops.FP8_K_PAD)
            return ops.linear_fp8(q, sx, layer.w_fp8, layer.w_scale, layer.bias, x0=x0, xl=xl)
        return ops.cross_v2(x0, xl, layer.weight, layer.bias)

    # (no resolve lane: the fp8 gather of step k+1 on the aux lane beside step
    # k's cross GEMMs measured no gain, 26.86 / 26.85 vs 27.13 / 26.99 M
    # one-stream, profiles/r04_session2.md - the cross GEMMs hold every CU;
    # the hooks were removed in round 5)

    def _front(self, ids, wts):
        """x0 and (fp8 towers) its e4m3 copy + row scales. x0 is quantised once,
        for the first cross layer AND the first MLP layer (both read it) - by
        the gather itself, which holds each row in one wave's registers
        (ops.embed_fp8; no separate quant pass)."""
        fp8_full = self.fp8 and not self.low_rank
        if fp8_full and self.cfg.num_fields <= 64:
            x0, *q0 = ops.embed_fp8(self.emb, ids, wts, self.cfg.vocab_size, ops.FP8_K_PAD)
            return x0, tuple(q0)
        x0, _ = ops.embed(self.emb, ids, wts, modulo=self.cfg.vocab_size, want_x=True)
        return x0, (ops.quant_rows_fp8(x0, ops.FP8_K_PAD) if fp8_full else None)

    def _cross_net(self, x0, q0):
        """The cross layers -> the cross half of the head logit."""
        fp8_full = self.fp8 and not self.low_rank
        L = self.cfg.num_cross_layers
        if fp8_full and self.d % 8 == 0 and L > 0:
            # split cross layers: plain-epilogue GEMM y = xl W^T + b (the
            # 8-phase tile runs it) + one combine pass that writes z = x0*y + xl,
            # quantises it for the next layer and, for the last layer, reduces
            # the cross logit instead of writing z (profiles/dcn_v2_split_kernels.md)
            # Full-chip steps: the combine rides on the GEMM as an LDS-staged
            # epilogue (ops.cross_gemm_fp8; no y round trip), the last layer
            # writing only per-column-tile partial cross logits; z is quantised
            # for the next layer by one quant_rows pass (it reads z back from
            # the Infinity Cache: cheaper than an e4m3 copy from the epilogue,
            # profiles/r03_cross_fused.md)
            xl, (q, sx) = x0, q0
            fused = ops.cross_gemm_fits(x0.shape[0], self.d) and q.shape[1] % 128 == 0
            for i in range(L):
                layer = self.cross[i]
                last = i == L - 1
                if fused:
                    z, cross_logit = ops.cross_gemm_fp8(q, sx, layer.w_fp8, layer.w_scale, layer.bias, x0, xl,
                                                        want_z=not last, head_w=self.head_wc if last else None)
                    if not last:
                        q, sx = ops.quant_rows_fp8(z, ops.FP8_K_PAD)
                else:
                    y = ops.linear_fp8(q, sx, layer.w_fp8, layer.w_scale, layer.bias)  # plain bf16 epilogue
                    z, q, sx, cross_logit = ops.cross_combine(y, x0, xl, want_z=not last,
                                                              k_pad=0 if last else ops.FP8_K_PAD,
                                                              head_w=self.head_wc if last else None)
                xl = z
            return cross_logit
        xl, xq = x0, q0
        for i in range(L):
            xl, xq = self._cross_layer(i, x0, xl, xq), None
        return ops.head(xl, self.head_wc, 0.0, sigmoid=False)

    def _mlp_q(self, x0, q0):
        return q0 if (q0 is not None and self.mlp.layers[0].fp8 and self.mlp.layers[0].k == x0.shape[1]) else None

    def _forward(self, ids, wts, out=None, resolved=None):
        x0, q0 = self._front(ids, wts)
        cross_logit = self._cross_net(x0, q0)
        return self.mlp.forward_head(x0, self.head_wd, self.head_b, extra=cross_logit, out=out, xq=self._mlp_q(x0, q0))

    # (not adopted, round 6: the first MLP layer on a step program's aux lane
    # beside the cross layers, to fill the CUs the cross GEMMs' last tile round
    # leaves idle - 27.86 / 28.05 / 27.49 M with the aux lane on 128 / all / 64
    # CUs vs 27.78 M one-lane, profiles/r06_dcn_mlp_lane.jsonl)


class DLRM(CTRModel):
    """DLRM: bottom MLP on dense fields, one table per sparse field, pairwise dot
    interaction (K5, MFMA), top MLP. ``table_shards`` restricts the tables this
    process materialises (embedding model parallelism, see parallel/)."""

    family = "dlrm"

    def __init__(self, cfg: ModelConfig, device="cpu", materialize_tables: bool = True):
        super().__init__(cfg, device)
        D, T = cfg.embed_dim, cfg.num_sparse
        assert D == 64, "DLRM dot-interaction kernel is built for D = 64"
        assert cfg.bottom_mlp[-1] == D, "bottom MLP must end at the embedding dim"
        self.T = T
        # dense features zero padded to one 128-byte K tile: the bottom MLP's
        # first GEMM takes the LDS-DMA kernel, not the register-staged fallback
        self.dense_k = -(-cfg.num_dense // 64) * 64
        self.bottom = MLP(cfg.num_dense, cfg.bottom_mlp, self.dtype, self.device_, self.gen, in_pad=self.dense_k)
        self.inter_cols = ops.interaction_cols(T, D)
        self.top = MLP(self.inter_cols, cfg.mlp_dims, self.dtype, self.device_, self.gen)
        self.head_w = nn.Parameter(init_uniform_(torch.empty(self.top.out_dim, device=self.device_), 0.05, self.gen),
                                   requires_grad=False)
        self.head_b = 0.0
        rows = cfg.table_rows
        self.hot = max(1, int(cfg.multi_hot))
        if cfg.num_dense + T * self.hot != cfg.num_fields:
            raise ValueError(f"dlrm: {cfg.num_fields} fields != {cfg.num_dense} dense + {T} tables x {self.hot} ids")
        self.register_buffer("modulo_f", torch.full((T,), rows, dtype=torch.int64, device=self.device_),
                             persistent=False)
        self.register_buffer("offset_f", torch.arange(T, dtype=torch.int64, device=self.device_) * rows,
                             persistent=False)
        # multi-hot: per id column (table t owns columns t*hot .. t*hot + hot - 1)
        self.register_buffer("col_mod", self.modulo_f.repeat_interleave(self.hot), persistent=False)
        self.register_buffer("col_off", self.offset_f.repeat_interleave(self.hot), persistent=False)
        self.emb = None
        if materialize_tables:
            t = torch.empty(T * rows, D, dtype=self.dtype, device=self.device_)
            for f in range(T):  # per-table hashed init: shards built elsewhere match these rows exactly
                hashed_uniform_rows_(t[f * rows:(f + 1) * rows], f, 0, cfg.seed, self.table_bound)
            self.emb = nn.Parameter(t, requires_grad=False)

    @property
    def table_bound(self) -> float:
        return 1.0 / math.sqrt(self.cfg.embed_dim)

    def dense_input(self, wts: torch.Tensor) -> torch.Tensor:
        """Dense features (the first num_dense weight columns) as the bottom
        MLP's zero-padded bf16 input [B, dense_k]: one kernel on the GPU."""
        nd = self.cfg.num_dense
        if wts.is_cuda and wts.dtype == torch.float32 and self.dtype == torch.bfloat16 and wts.stride(1) == 1:
            return ops.hip().dense_pad(wts, nd, self.dense_k)
        x = torch.zeros(wts.shape[0], self.dense_k, dtype=self.dtype, device=wts.device)
        x[:, :nd] = wts[:, :nd]
        return x

    def sparse_ids(self, ids: torch.Tensor) -> torch.Tensor:
        """The sparse id columns as a row view (the gather kernels take a row
        stride; a .contiguous() copy here was a 9 us kernel per served step)."""
        return ids[:, self.cfg.num_dense:]

    def lookup(self, ids: torch.Tensor, wts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Local (single-process) lookup of every sparse table -> [B, T, D].
        One-hot: the K1 gather. Multi-hot (``cfg.multi_hot`` ids per table):
        ids hashed onto global table rows (K0), then the K1b bag kernel sums
        each table's ``hot`` rows weighted by their feat_wts."""
        B = ids.shape[0]
        sp = self.sparse_ids(ids)
        if self.hot == 1:
            x, _ = ops.embed(self.emb, sp, None, modulo_f=self.modulo_f, offset_f=self.offset_f, want_x=True)
            return x.view(B, self.T, self.cfg.embed_dim)
        rows = ops.pack_ids(sp, modulo_f=self.col_mod, offset_f=self.col_off)  # int32 [B, T*hot]
        w = None
        if wts is not None:
            w = wts[:, self.cfg.num_dense:].float().contiguous().view(-1)
        offsets = torch.arange(0, B * self.T * self.hot + 1, self.hot, dtype=torch.int64, device=rows.device)
        pooled = ops.embedding_bag(self.emb, rows.view(-1), offsets, per_sample_weights=w, out_bf16=True)
        return pooled.view(B, self.T, self.cfg.embed_dim)

    def interact_and_top(self, dense_out: torch.Tensor, emb: torch.Tensor, out=None) -> torch.Tensor:
        z = ops.dot_interaction(dense_out, emb, self.inter_cols)
        return self.top.forward_head(z, self.head_w, self.head_b, out=out)

    def _bottom_fused(self) -> bool:
        L = self.bottom.layers
        return (self.dtype == torch.bfloat16 and self.dense_k == 64
                and tuple(l.out_dim for l in L) == ops.BOTTOM_MLP3_DIMS and all(l.act == "relu" for l in L)
                and not any(l.fp8 for l in L))

    def bottom_out(self, wts) -> torch.Tensor:
        """Bottom MLP over the dense features: one fused kernel on the GPU for
        the 512-256-64 tower (pad + 3 GEMMs were ~31 us of mostly launch /
        prologue per 16384-row step), else layer by layer. ``wts`` may be
        :class:`ops.ArenaRows` (fused path only)."""
        L = self.bottom.layers
        if isinstance(wts, ops.ArenaRows) or (wts.is_cuda and wts.dtype == torch.float32 and self._bottom_fused()):
            return ops.bottom_mlp3(wts, self.cfg.num_dense, [(l.weight, l.bias) for l in L])
        return self.bottom(self.dense_input(wts))

    def narrow_weight_cols(self) -> int:
        """Leading feat_wts columns the forward reads: one-hot DLRM reads only
        the dense features (its sparse lookups are unweighted), so host-narrowed
        requests carry just those (serving/live.py); 0 = all."""
        return self.cfg.num_dense if self.hot == 1 else 0

    @property
    def supports_arena(self) -> bool:
        """One-hot, local tables, the fused bottom tower: the step reads the
        request arena itself (no unpack pass: K0 fused into the bottom MLP
        and the interaction's gather)."""
        return self.hot == 1 and self.emb is not None and self._bottom_fused()

    # (no resolve lane: step k+1's bottom MLP + gathered interaction on the
    # aux lane beside step k's top MLP measured slower, 100.2 / 100.5 vs
    # 106.1 / 107.0 M one-stream, profiles/r04_session2.md; hooks removed in
    # round 5)

    def _forward(self, ids, wts, out=None, resolved=None):
        arena = isinstance(ids, ops.ArenaRows)
        dense_out = self.bottom_out(ids if arena else wts)
        if self.hot == 1 and self.emb is not None and (arena or ids.is_cuda):
            # one-hot, local tables: the interaction kernel looks the rows up
            # itself (no [B, T, 64] embedding round trip through HBM)
            z = ops.dot_interaction_gather(dense_out, self.emb, ids if arena else self.sparse_ids(ids), self.modulo_f,
                                           self.offset_f, self.inter_cols, id_col0=self.cfg.num_dense)
            return self.top.forward_head(z, self.head_w, self.head_b, out=out)
        emb = self.lookup(ids, wts)
        return self.interact_and_top(dense_out, emb, out=out)


FAMILIES = {c.family: c for c in (WideDeep, DeepFM, DCN, DCNv2, DLRM)}


def build_model(cfg: ModelConfig, device="cpu", **kw) -> CTRModel:
    try:
        cls = FAMILIES[cfg.family]
    except KeyError:
        raise ValueError(f"unknown model family {cfg.family!r}; known: {sorted(FAMILIES)}") from None
    m = cls(cfg, device=device, **kw).eval()
    m.gen = None  # init-only RNG; keeps the module deep-copyable / movable
    return m

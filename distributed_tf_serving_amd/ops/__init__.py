"""CTR compute ops: gfx950 HIP kernels for GPU tensors, reference math on CPU.

Every op dispatches on the device of its inputs:

* GPU tensor -> the hand-written CDNA4 kernel in ``csrc/kernels`` (through the
  ``_hip`` extension). There is no silent eager fallback: a missing extension
  raises (see :mod:`._loader`).
* CPU tensor -> the reference implementation in plain PyTorch (fp32 math).
  This is both the CPU serving backend and the numerics oracle the GPU tests
  compare against.

Op inventory: K0 ``pack_ids``, K1 ``embed``, K1b
``embedding_bag``, K2 FM (fused in ``embed``), K3 ``cross_v1``, K3b
``cross_v2`` / ``linear_fp8``, K4 ``linear``, K5 ``dot_interaction``, K6
``head``, K4+K6 ``linear_head``, K7 ``sort_scores``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ._loader import hip, hip_loaded, native  # noqa: F401

_ACTS = {"none": 0, "relu": 1, "sigmoid": 2}

FP8_MAX = 448.0  # OCP e4m3fn


def _hash_rows(ids: torch.Tensor, modulo: int = 0, modulo_f=None, offset_f=None) -> torch.Tensor:
    ids = ids.long()
    if modulo_f is not None:
        return offset_f.view(1, -1).to(ids.device) + torch.remainder(ids, modulo_f.view(1, -1).to(ids.device))
    if modulo and modulo > 0:
        return torch.remainder(ids, modulo)
    return ids


def _rows(t: torch.Tensor) -> torch.Tensor:
    """Row views with unit inner stride pass through (kernels take a row stride)."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t
    return t.contiguous()


# ------------------------------------------------------------------ K0
def pack_ids(ids: torch.Tensor, modulo: int = 0, modulo_f=None, offset_f=None) -> torch.Tensor:
    """int64/int32 feature ids -> int32 table rows (``offset_f + id mod m``)."""
    if ids.is_cuda:
        return hip().pack_ids(ids.contiguous(), int(modulo), modulo_f, offset_f)
    return _hash_rows(ids, modulo, modulo_f, offset_f).to(torch.int32)


@dataclass(frozen=True)
class ArenaRows:
    """Candidate rows still inside a request arena (serving/arena.py): passed
    as ``ids`` to :func:`embed`, the gather reads each row's ids and weights
    from the raw request bytes (K0 fused into K1)."""

    arena: torch.Tensor  # uint8 arena (device for the kernel, host for the reference)
    B: int
    F: int

    @property
    def shape(self):
        return (self.B, self.F)


def _arena_unpack_host(rows: "ArenaRows") -> Tuple[torch.Tensor, torch.Tensor]:
    from ..serving.packing import PackedLayout

    L = PackedLayout(rows.F)
    packed = L.alloc(rows.B)
    native().arena_unpack_cpu(rows.arena.cpu().contiguous(), packed, rows.F)
    return L.ids(packed), L.wts(packed)


# ------------------------------------------------------------------ K1 (+K2)
def embed(table: torch.Tensor, ids: torch.Tensor, wts: Optional[torch.Tensor] = None,
          lin: Optional[torch.Tensor] = None, modulo: int = 0, modulo_f=None, offset_f=None,
          bias: float = 0.0, want_x: bool = True, want_fm: bool = False, fm2: bool = False,
          out_x: Optional[torch.Tensor] = None, shard_lo_f: Optional[torch.Tensor] = None,
          shard_n_f: Optional[torch.Tensor] = None) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Weighted embedding gather with fused factorisation-machine terms.

    x[b, f*D:(f+1)*D] = table[row(b, f)] * wts[b, f]
    fm[b] = bias + sum_f lin[row]*wts  (if lin) + 0.5*sum_d((sum_f e)^2 - sum_f e^2)  (if fm2)

    ``shard_lo_f``/``shard_n_f`` (row-wise sharded tables): field f's table
    here holds global rows [lo, lo + n) at ``offset_f[f]``; ids hashing
    elsewhere contribute zeros.

    ``ids`` may be :class:`ArenaRows` (then ``wts`` is None): rows come from
    the raw request bytes of a request arena.
    """
    if isinstance(ids, ArenaRows):
        if modulo_f is not None or shard_lo_f is not None:
            raise ValueError("arena rows support the shared-table gather only")
        if ids.arena.is_cuda:
            m = int(modulo) if modulo > 0 else table.shape[0]
            x, fm, _, _ = hip().embed_arena(table, lin, ids.arena, int(ids.B), int(ids.F), m, float(bias), want_x,
                                            want_fm, fm2, out_x)
            return (x if want_x else None), (fm if want_fm else None)
        ids, wts = _arena_unpack_host(ids)
    if ids.is_cuda:
        if modulo_f is None and modulo <= 0:
            modulo = table.shape[0]
        x, fm, _, _ = hip().embed(table, lin, _rows(ids), None if wts is None else _rows(wts), int(modulo),
                            modulo_f, offset_f, float(bias), want_x, want_fm, fm2, out_x, False, shard_lo_f, shard_n_f)
        return (x if want_x else None), (fm if want_fm else None)
    if shard_lo_f is not None:
        g = torch.remainder(ids.long(), modulo_f.view(1, -1)) - shard_lo_f.view(1, -1)
        own = (g >= 0) & (g < shard_n_f.view(1, -1))
        rows = offset_f.view(1, -1) + torch.where(own, g, torch.zeros_like(g))
        w_own = own.float() if wts is None else wts.float() * own
        wts = w_own
    else:
        rows = _hash_rows(ids, modulo if modulo > 0 else table.shape[0], modulo_f, offset_f)
    e = table[rows].float()  # [B, F, D]
    if wts is not None:
        e = e * wts.float().unsqueeze(-1)
    x = None
    if want_x:
        x = e.reshape(e.shape[0], -1).to(table.dtype)
        if out_x is not None:
            out_x.copy_(x.view_as(out_x))
            x = out_x
    fm = None
    if want_fm:
        fm = torch.full((ids.shape[0],), float(bias), dtype=torch.float32)
        if lin is not None:
            w1 = lin[rows].float()
            fm = fm + (w1 * (wts.float() if wts is not None else 1.0)).sum(1)
        if fm2:
            s = e.sum(1)
            fm = fm + 0.5 * (s * s - (e * e).sum(1)).sum(1)
    return x, fm


# ------------------------------------------------------------------ K1b
def embed_fp8(table: torch.Tensor, ids, wts: Optional[torch.Tensor], modulo: int, k_pad: int):
    """Weighted gather that also returns x as the fp8 towers' first operand:
    (x bf16 [B, F*D], q e4m3 [B, K padded to k_pad], per-row scale [B]) - the
    same values as ``quant_rows_fp8(x, k_pad)``, written by the gather itself
    (shared-table gather, F <= 64)."""
    m = int(modulo) if modulo > 0 else table.shape[0]
    if isinstance(ids, ArenaRows):
        if ids.arena.is_cuda:
            x, _, q, s = hip().embed_arena(table, None, ids.arena, int(ids.B), int(ids.F), m, 0.0, True, False,
                                           False, None, int(k_pad))
            return x, q, s
    elif ids.is_cuda:
        x, _, q, s = hip().embed(table, None, _rows(ids), None if wts is None else _rows(wts), m,
                                 None, None, 0.0, True, False, False, None, False, None, None, int(k_pad))
        return x, q, s
    x, _ = embed(table, ids, wts, modulo=m, want_x=True)
    q, s = quant_rows_fp8(x, k_pad)
    return x, q, s


def embedding_bag(table: torch.Tensor, indices: torch.Tensor, offsets: torch.Tensor,
                  per_sample_weights: Optional[torch.Tensor] = None, modulo: int = 0, mean: bool = False,
                  out_bf16: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sum (or mean) pooled multi-hot lookup; offsets are CSR [nbags + 1].
    ``out``: a static [nbags, D] buffer to write (captured steps)."""
    if table.is_cuda:
        m = int(modulo) if modulo > 0 else table.shape[0]
        return hip().embedding_bag(table, indices.contiguous(), offsets.contiguous(), per_sample_weights, m, mean,
                                   out_bf16, out)
    rows = _hash_rows(indices, modulo if modulo > 0 else table.shape[0])
    res = torch.nn.functional.embedding_bag(rows, table.float(), offsets[:-1], mode="mean" if mean else "sum",
                                            per_sample_weights=None if mean else per_sample_weights,
                                            include_last_offset=False)
    if mean and per_sample_weights is not None:
        raise ValueError("per_sample_weights with mean pooling is not supported")
    res = res.to(torch.bfloat16) if out_bf16 else res
    if out is not None:
        out.copy_(res.view(out.shape))
        return out
    return res


# ------------------------------------------------------------------ K4 / K3b
def linear(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None, act: str = "none",
           out_f32: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(x W^T + b) on MFMA (bf16 in, fp32 accumulate, bf16/fp32 out)."""
    if x.is_cuda:
        return hip().gemm(x, W, b, _ACTS[act], None, None, out_f32, None, None, out)
    y = x.float() @ W.float().t()
    if b is not None:
        y = y + b.float()
    if act == "relu":
        y = torch.relu(y)
    elif act == "sigmoid":
        y = torch.sigmoid(y)
    y = y if out_f32 else y.to(x.dtype if x.dtype != torch.float32 else torch.float32)
    if out is not None:
        out.copy_(y)
        return out
    return y


def cross_v2(x0: torch.Tensor, xl: torch.Tensor, W: torch.Tensor, b: torch.Tensor,
             a: Optional[torch.Tensor] = None) -> torch.Tensor:
    """DCN-v2 cross layer x0 * (a W^T + b) + xl, fused in the GEMM epilogue.

    ``a`` defaults to ``xl`` (full rank); the low-rank form passes a = V xl."""
    a = xl if a is None else a
    if x0.is_cuda:
        return hip().gemm(a, W, b, 3, x0, xl, False, None, None, None)
    y = a.float() @ W.float().t() + b.float()
    return (x0.float() * y + xl.float()).to(x0.dtype)


FP8_K_PAD = 128  # K granularity of the block-scaled fp8 MFMA (16x16x128) tiles


def quant_rows_fp8(x: torch.Tensor, k_pad: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Dynamic per-row OCP e4m3 quantisation: (q, scale) with x ~= q * scale.

    ``k_pad``: q's row width is K rounded up to it, zero-filled (fp8 GEMM
    operands use FP8_K_PAD so every K tile is a full 128-deep MFMA)."""
    if x.is_cuda:
        return tuple(hip().quant_rows_fp8(_rows(x), int(k_pad)))
    xf = x.float()
    amax = xf.abs().amax(dim=1).clamp_min(0)
    scale = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    q = (xf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    Kq = -(-x.shape[1] // k_pad) * k_pad
    if Kq != x.shape[1]:
        q = torch.cat([q, torch.zeros(x.shape[0], Kq - x.shape[1], dtype=q.dtype)], dim=1)
    return q, scale


MX_BLOCK = 32  # OCP MX: one E8M0 scale per 32 consecutive K elements
MX_MAX_K = 3072  # MX-scaled GEMM input: the block's scale panel is staged in LDS


def _mx_exponent(amax: torch.Tensor) -> torch.Tensor:
    """Smallest e with amax / 2^e <= FP8_MAX (0 for an all-zero block)."""
    m, ex = torch.frexp(amax / FP8_MAX)
    e = torch.where(m == 0.5, ex - 1, ex)
    return torch.where(amax > 0, e, torch.zeros_like(e)).clamp(-127, 127)


def quant_mx_fp8(x: torch.Tensor, k_pad: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """OCP MX-fp8 quantisation of rows (CPU reference of the GEMM epilogue that
    emits it): q e4m3 [M, Kq] and E8M0 scale bytes [M, Kq / 32] with
    x ~= q * 2^(scale - 127) per 32-column block; K padding is zero (scale 127)."""
    M, K = x.shape
    Kq = -(-K // max(k_pad, MX_BLOCK)) * max(k_pad, MX_BLOCK)
    xf = torch.zeros(M, Kq, dtype=torch.float32, device=x.device)
    xf[:, :K] = x.float()
    blk = xf.view(M, Kq // MX_BLOCK, MX_BLOCK)
    e = _mx_exponent(blk.abs().amax(dim=2))
    q = (blk * torch.exp2(-e.float())[:, :, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn)
    return q.view(M, Kq), (e + 127).to(torch.uint8)


def dequant_mx_fp8(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    return q.float() * torch.exp2(s.float() - 127).repeat_interleave(MX_BLOCK, dim=1)


def cross_combine(y: torch.Tensor, x0: torch.Tensor, xl: torch.Tensor, want_z: bool = True, k_pad: int = 0,
                  head_w: Optional[torch.Tensor] = None):
    """Split DCN-v2 cross layer, second half: z = x0 * y + xl (bf16), in one pass
    over the rows also quantised (``k_pad`` > 0: e4m3 + per-row scale, zero
    padded to a multiple of k_pad - the next layer's fp8 operand) and/or dotted
    with ``head_w`` (the last layer's cross logit). Returns (z, q, scale, dot),
    None for what was not asked."""
    if y.is_cuda:
        z, q, s, d = hip().cross_combine(y.contiguous(), x0.contiguous(), xl.contiguous(), want_z, int(k_pad),
                                         head_w)
        return (z if want_z else None, q if k_pad else None, s if k_pad else None,
                d if head_w is not None else None)
    zb = (x0.float() * y.float() + xl.float()).to(torch.bfloat16)
    q = s = d = None
    if k_pad:
        q, s = quant_rows_fp8(zb, k_pad)
    if head_w is not None:
        d = zb.float() @ head_w.float()
    return (zb if want_z else None, q, s, d)


CROSS_TILE = 256  # column tile of the fused cross GEMM: one partial logit per tile


def cross_gemm_fits(M: int, N: int) -> bool:
    """The fused cross GEMM runs 256x256 tiles: worth it once they fill the chip
    (smaller steps take linear_fp8 + cross_combine on smaller tiles)."""
    return -(-M // 256) * -(-N // 256) >= 256 and N % 8 == 0




def cross_gemm_fp8(xq: torch.Tensor, sx: torch.Tensor, Wq: torch.Tensor, sw: torch.Tensor,
                   b: Optional[torch.Tensor], x0: torch.Tensor, xl: torch.Tensor, want_z: bool = True,
                   head_w: Optional[torch.Tensor] = None):
    """One DCN-v2 cross layer in one launch (csrc/kernels/gemm.hip
    cross_staged_epilogue): y = bf16(xq Wq^T * sx * sw + b), z = bf16(x0 * y + xl).
    Returns (z or None, dot or None) with dot = fp32 [tiles, M] partial cross
    logits z[:, T t:T t + T] . head_w[T t:T t + T] (a head ``extra``; T = 256).
    The same rounding as linear_fp8 + cross_combine."""
    if xq.is_cuda:
        z, d = hip().cross_gemm_fp8(xq, sx, Wq, sw, b, x0, xl, want_z, head_w)
        return (z if want_z else None), (d if head_w is not None else None)
    y = linear_fp8(xq, sx, Wq, sw, b)
    zb = (x0.float() * y.float() + xl.float()).to(torch.bfloat16)
    d = None
    if head_w is not None:
        N = zb.shape[1]
        d = torch.stack([zb[:, t:t + CROSS_TILE].float() @ head_w[t:t + CROSS_TILE].float()
                         for t in range(0, N, CROSS_TILE)])
    return (zb if want_z else None), d


def linear_fp8(xq: torch.Tensor, sx: Optional[torch.Tensor], Wq: torch.Tensor, sw: torch.Tensor,
               b: Optional[torch.Tensor] = None, act: str = "none", out_f32: bool = False,
               x0: Optional[torch.Tensor] = None, xl: Optional[torch.Tensor] = None,
               sx_blk: Optional[torch.Tensor] = None, emit_mx: int = 0):
    """fp8 x fp8 -> fp32-accumulated GEMM with row/channel scales (CDNA4 fp8 MFMA).

    ``x0``/``xl`` given selects the DCN-v2 cross epilogue.
    ``sx_blk``: MX block scales of xq (uint8 E8M0 [M, K/32]) applied by the MFMA
    itself, instead of (or on top of) the row scales ``sx``.
    ``emit_mx = nq > 0`` (cross epilogue only): the epilogue also writes its
    output as the next GEMM's MX-fp8 operand; returns (y, q [M, nq], scales
    [M, nq/32])."""
    epi = 3 if x0 is not None else _ACTS[act]
    if emit_mx and epi != 3:
        raise ValueError("emit_mx needs the cross epilogue")
    if xq.is_cuda:
        if emit_mx:
            M = xq.shape[0]
            q = torch.empty(M, emit_mx, dtype=torch.float8_e4m3fn, device=xq.device)
            sq = torch.empty(M, emit_mx // MX_BLOCK, dtype=torch.uint8, device=xq.device)
            y = hip().gemm(xq, Wq, b, epi, x0, xl, out_f32, sx, sw, None, 0, sx_blk, q, sq)
            return y, q, sq
        return hip().gemm(xq, Wq, b, epi, x0, xl, out_f32, sx, sw, None, 0, sx_blk)
    xf = dequant_mx_fp8(xq, sx_blk) if sx_blk is not None else xq.float()
    if sx is not None:
        xf = xf * sx[:, None]
    y = xf @ (Wq.float() * sw[:, None]).t()
    if b is not None:
        y = y + b.float()
    if epi == 3:
        y = x0.float() * y + xl.float()
    elif act == "relu":
        y = torch.relu(y)
    elif act == "sigmoid":
        y = torch.sigmoid(y)
    out = y if out_f32 else y.to(torch.bfloat16)
    if emit_mx:
        return (out,) + quant_mx_fp8(y, emit_mx)
    return out


# ------------------------------------------------------------------ K3
def cross_v1(x0: torch.Tensor, w: torch.Tensor, b: torch.Tensor, want_x: bool = True,
             head_w: Optional[torch.Tensor] = None):
    """DCN cross network, all layers: x_{l+1} = x0 * (x_l . w_l) + b_l + x_l.

    Returns (x_L or None, x_L . head_w or None)."""
    if x0.is_cuda:
        x, d = hip().cross_v1(x0.contiguous(), w, b, want_x, head_w)
        return (x if want_x else None), (d if head_w is not None else None)
    a0 = x0.float()
    xl = a0
    for l in range(w.shape[0]):
        s = xl @ w[l].float()
        xl = a0 * s[:, None] + b[l].float() + xl
    dot = (xl @ head_w.float()) if head_w is not None else None
    return (xl.to(x0.dtype) if want_x else None), dot


def cross_v1_consts(w: torch.Tensor, b: torch.Tensor, head_w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Weights of the DCN v1 cross network folded for the gather (K3 in K1,
    csrc/kernels/embedding.hip): (rows [w_0..w_{L-1}, head_w] fp32 [L+1, d],
    c [L+1] with c_l = (b_0 + .. + b_{l-1}) . w_l and c_L = (b_0 + .. + b_{L-1})
    . head_w). Per row the cross logit is then alpha_L (x0 . head_w) + c_L with
    alpha_0 = 1, alpha_{l+1} = alpha_l (1 + x0 . w_l) + c_l."""
    rows = torch.cat([w.float(), head_w.float().view(1, -1)], 0).contiguous()
    beta = torch.cumsum(torch.cat([torch.zeros_like(b[:1].float()), b.float()], 0), 0)  # beta_0 .. beta_L
    c = (beta * rows).sum(1).contiguous()
    return rows, c


def embed_cross(table: torch.Tensor, ids, wts: Optional[torch.Tensor], modulo: int, w: torch.Tensor,
                b: torch.Tensor, head_w: torch.Tensor, consts=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Weighted gather + the whole DCN v1 cross network: (x bf16 [B, F*D],
    cross logit x_L . head_w fp32 [B]). On the GPU one kernel (the gather wave
    holds x0; ``consts`` = cross_v1_consts(...), cached by the caller); on the
    CPU the layer-by-layer reference math."""
    m = int(modulo) if modulo > 0 else table.shape[0]
    on_gpu = ids.arena.is_cuda if isinstance(ids, ArenaRows) else ids.is_cuda
    if on_gpu:
        rows, c = consts if consts is not None else cross_v1_consts(w, b, head_w)
        if isinstance(ids, ArenaRows):
            x, logit, _, _ = hip().embed_arena(table, None, ids.arena, int(ids.B), int(ids.F), m, 0.0, True, True,
                                               False, None, 0, rows, c)
        else:
            x, logit, _, _ = hip().embed(table, None, _rows(ids), None if wts is None else _rows(wts), m, None, None,
                                         0.0, True, True, False, None, False, None, None, 0, rows, c)
        return x, logit
    x, _ = embed(table, ids, wts, modulo=m, want_x=True)
    _, logit = cross_v1(x, w, b, want_x=False, head_w=head_w)
    return x, logit


# ------------------------------------------------------------------ K1 fused into K4
# Below this many candidate rows the gather-GEMM's 256x256 tiles leave most
# CUs idle and the separate gather + smaller-tile GEMM wins (tools/studies/
# microbench.py --gather-gemm, profiles/r03_gather_gemm.md).
GATHER_GEMM_MIN_ROWS = 16384


def embed_gemm_ok(table: torch.Tensor, W: torch.Tensor, B: int, fm2: bool) -> bool:
    """Shapes the gather-GEMM covers: a bf16 [V, 64] table, a bf16 first layer
    with N % 256 == 0 (N >= 1024 with the FM term or the cross network), enough
    rows to fill the GPU."""
    N, K = W.shape
    return (table.is_cuda and table.dtype == torch.bfloat16 and table.dim() == 2 and table.shape[1] == 64
            and W.dtype == torch.bfloat16 and N % 256 == 0 and (not fm2 or N >= 1024)
            and table.shape[0] <= 2 ** 31 and N * K * 2 < 2 ** 31 and B >= GATHER_GEMM_MIN_ROWS)


def embed_gemm_resolve(table: torch.Tensor, ids, wts: Optional[torch.Tensor], lin: Optional[torch.Tensor],
                       modulo: int, bias: float, two_parts: bool) -> Tuple[torch.Tensor, ...]:
    """The gather-GEMM's front half alone (GPU): (rows_t, wts_t, parts) for
    ``embed_gemm(..., resolved=...)``, so a step program can resolve step k+1
    on its aux lane while the compute lane finishes step k. ``two_parts``: the
    consumer computes the FM term or the cross network (fm2 or cross)."""
    m = int(modulo) if modulo > 0 else table.shape[0]
    n_parts = 2 if two_parts else 1
    if isinstance(ids, ArenaRows):
        return tuple(hip().embed_gemm_resolve(table, lin, ids.arena, None, None, int(ids.B), int(ids.F), m,
                                              float(bias), n_parts))
    return tuple(hip().embed_gemm_resolve(table, lin, None, _rows(ids), None if wts is None else _rows(wts),
                                          int(ids.shape[0]), int(ids.shape[1]), m, float(bias), n_parts))


def embed_gemm(table: torch.Tensor, ids, wts: Optional[torch.Tensor], lin: Optional[torch.Tensor], modulo: int,
               bias: float, W: torch.Tensor, b: torch.Tensor, act: str = "relu",
               fm2: bool = True, cross=None, resolved=None, packed_w=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """K1 fused into the first MLP layer (K4): returns
      h     = act(x W^T + b) bf16 [B, N], x[b, 64f:64f+64] = bf16(T[row(b, f)] * w(b, f)),
      parts = fp32 [1 + fm2, >= B]: row 0 = bias + sum_f lin[row] w, row 1 the
              second-order FM term (heads sum the rows, _extra_logit).
    ``cross = (w, b, head_w)`` (DCN v1, fm2 False): row 1 of parts is the cross
    network's logit x_L . head_w instead (the GPU takes the folded weights,
    ``cross_consts = cross_v1_consts(w, b, head_w)``, as ``cross[3]`` when given).
    ``resolved``: the front half from :func:`embed_gemm_resolve` (GPU only).
    ``packed_w``: a callable returning W in 32x32x16 MFMA fragment order
    (:func:`pack_frag32`, e.g. ``lambda: dense.packed("32")``); with it (N % 512 ==
    0, no cross network) the GPU runs the one-wave-per-SIMD form
    (csrc/kernels/gather_gemm.hip: B straight into registers).
    On the GPU x never exists in HBM (csrc/kernels/gemm.hip gemm_gather_kernel reads
    table rows straight into the GEMM's LDS tiles); on the CPU the unfused math."""
    m = int(modulo) if modulo > 0 else table.shape[0]
    on_gpu = ids.arena.is_cuda if isinstance(ids, ArenaRows) else ids.is_cuda
    if on_gpu:
        a = _ACTS[act]
        xw = xc = None
        if cross is not None:
            xw, xc = cross[3] if len(cross) > 3 and cross[3] is not None else cross_v1_consts(*cross[:3])
        r = list(resolved) if resolved is not None else None
        wp = packed_w() if packed_w is not None and cross is None and W.shape[0] % 512 == 0 else None
        if isinstance(ids, ArenaRows):
            return tuple(hip().embed_gemm(table, lin, ids.arena, None, None, int(ids.B), int(ids.F), m, float(bias),
                                          W, b, a, fm2, xw, xc, r, wp))
        return tuple(hip().embed_gemm(table, lin, None, _rows(ids), None if wts is None else _rows(wts),
                                      int(ids.shape[0]), int(ids.shape[1]), m, float(bias), W, b, a, fm2, xw, xc, r,
                                      wp))
    if cross is not None:
        x, logit = embed_cross(table, ids, wts, m, cross[0], cross[1], cross[2])
        first = torch.full((1, x.shape[0]), float(bias), dtype=torch.float32)
        if lin is not None:
            _, fm = embed(table, ids, wts, lin=lin, modulo=m, bias=bias, want_x=False, want_fm=True, fm2=False)
            first = fm.view(1, -1)
        return linear(x, W, b, act), torch.cat([first, logit.float().view(1, -1)])
    x, fm = embed(table, ids, wts, lin=lin, modulo=m, bias=bias, want_x=True, want_fm=True, fm2=fm2)
    return linear(x, W, b, act), fm.view(1, -1)


# ------------------------------------------------------------------ K5
def interaction_cols(num_sparse: int, dim: int = 64) -> int:
    """Width of the interaction output (and the top MLP's K), zero padded to a
    multiple of 64: the top MLP's first GEMM then reads whole 128-byte K tiles
    (LDS-DMA / 8-phase kernels) instead of the register-staged fallback."""
    used = dim + (num_sparse + 1) * num_sparse // 2
    return (used + 63) // 64 * 64


def dot_interaction(dense: torch.Tensor, emb: torch.Tensor, out_cols: int = 0,
                    emb_off: Optional[torch.Tensor] = None, emb_stride: Optional[torch.Tensor] = None) -> torch.Tensor:
    """DLRM: [dense | strictly-lower-triangular entries of X X^T | zero pad], X = [dense; emb].

    ``emb`` is [B, T, D], or with a table map (``emb_off`` / ``emb_stride``,
    int64 [T]) a flat [N, D] buffer in which table t of row b is row
    ``emb_off[t] + b * emb_stride[t]`` - the layout an embedding all-to-all
    leaves behind, read in place (parallel/embedding_sharding.py)."""
    mapped = emb_off is not None
    T = int(emb_off.numel()) if mapped else emb.shape[1]
    if out_cols <= 0:
        out_cols = interaction_cols(T, dense.shape[1])
    if dense.is_cuda:
        if mapped:
            return hip().dot_interaction(dense.contiguous(), emb, int(out_cols), emb_off, emb_stride)
        return hip().dot_interaction(dense.contiguous(), emb.contiguous(), int(out_cols))
    if mapped:
        rows = emb_off.view(1, -1) + torch.arange(dense.shape[0]).view(-1, 1) * emb_stride.view(1, -1)
        emb = emb[rows.clamp(0, emb.shape[0] - 1)]  # [B, T, D]
    X = torch.cat([dense.float().unsqueeze(1), emb.float()], dim=1)  # [B, T+1, D]
    Z = X @ X.transpose(1, 2)
    li, lj = torch.tril_indices(T + 1, T + 1, offset=-1)
    out = torch.zeros(dense.shape[0], out_cols, dtype=torch.float32)
    out[:, : dense.shape[1]] = dense.float()
    out[:, dense.shape[1]: dense.shape[1] + li.numel()] = Z[:, li, lj]
    return out.to(dense.dtype)


def dot_interaction_gather(dense: torch.Tensor, table: torch.Tensor, ids, modulo_f: torch.Tensor,
                           offset_f: torch.Tensor, out_cols: int = 0, id_col0: int = 0) -> torch.Tensor:
    """K1 fused into K5 (one-hot DLRM, local tables): dot_interaction(dense,
    table[offset_f + ids mod modulo_f]) without the [B, T, 64] embedding
    intermediate. ``ids``: int32/int64 [B, T] rows (a row view is fine), or
    :class:`ArenaRows` whose features id_col0 .. id_col0 + T - 1 are the ids."""
    T = int(modulo_f.numel())
    if out_cols <= 0:
        out_cols = interaction_cols(T, dense.shape[1])
    if isinstance(ids, ArenaRows):
        if ids.arena.is_cuda:
            return hip().dot_interaction_gather_arena(dense, table, ids.arena, int(id_col0), modulo_f, offset_f,
                                                      int(out_cols))
        ids = _arena_unpack_host(ids)[0][:, id_col0:id_col0 + T]
    if dense.is_cuda:
        return hip().dot_interaction_gather(dense, table, _rows(ids), modulo_f, offset_f, int(out_cols))
    rows = _hash_rows(ids, 0, modulo_f, offset_f).clamp(0, table.shape[0] - 1)
    return dot_interaction(dense, table[rows], out_cols)


def dot_interaction_gather_peer(dense: torch.Tensor, ids, peer, cache=None, out_cols: int = 0,
                                id_col0: int = 0) -> torch.Tensor:
    """K1 + K5 through the peer lookup (parallel/hot_cache.py): table t's row
    of candidate b is read where it lives - this rank's store, the owner's
    store over xGMI, or this rank's replica cache of hot remote rows. ``ids``:
    int32/int64 [B, >= id_col0 + T] rows or :class:`ArenaRows`."""
    T = peer.T
    if out_cols <= 0:
        out_cols = interaction_cols(T, dense.shape[1])
    kw = cache.kernel_args() if cache is not None else {}
    if dense.is_cuda:
        if isinstance(ids, ArenaRows):
            return hip().dot_interaction_gather_peer(dense, None, ids.arena, int(id_col0), out_cols=int(out_cols),
                                                     **peer.kernel_args(), **kw)
        return hip().dot_interaction_gather_peer(dense, _rows(ids), None, int(id_col0), out_cols=int(out_cols),
                                                 **peer.kernel_args(), **kw)
    from ..parallel.hot_cache import peer_gather_cpu

    if isinstance(ids, ArenaRows):
        ids = _arena_unpack_host(ids)[0]
    emb = peer_gather_cpu(peer, cache, ids[:, id_col0:id_col0 + T], None, 1)
    return dot_interaction(dense, emb, out_cols)


def peer_bag(ids, wts: Optional[torch.Tensor], B: int, col0: int, hot: int, peer, cache=None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K1b through the peer lookup: bf16 [B, T, 64] pooled bags (table t's bag =
    columns col0 + t * hot .. + hot - 1 of ``ids`` / ``wts``, or of the
    :class:`ArenaRows`)."""
    T = peer.T
    dev = peer.trows.device
    if out is None:
        out = torch.empty(B, T, 64, dtype=peer.dtype, device=dev)
    kw = cache.kernel_args() if cache is not None else {}
    if dev.type == "cuda":
        if isinstance(ids, ArenaRows):
            hip().peer_bag(None, None, ids.arena, int(B), int(col0), int(hot), out=out, **peer.kernel_args(), **kw)
        else:
            hip().peer_bag(_rows(ids), _rows(wts.float()), None, int(B), int(col0), int(hot), out=out,
                           **peer.kernel_args(), **kw)
        return out
    from ..parallel.hot_cache import peer_gather_cpu

    if isinstance(ids, ArenaRows):
        ids, wts = _arena_unpack_host(ids)
    n = T * hot
    out.copy_(peer_gather_cpu(peer, cache, ids[:, col0:col0 + n], wts[:, col0:col0 + n], hot).view_as(out))
    return out


BOTTOM_MLP3_DIMS = (512, 256, 64)  # the fused DLRM bottom-MLP kernel's layer widths


def bottom_mlp3(wts: torch.Tensor, nd: int, layers) -> torch.Tensor:
    """DLRM bottom MLP in one kernel (csrc/kernels/interaction.hip
    bottom_mlp3_kernel): relu layers 64 -> 512 -> 256 -> 64 over the fp32 dense
    feature columns wts[:, :nd] (bf16, zero padded to 64). ``layers``: three
    (weight bf16 [N, K], bias fp32 [N]) pairs. bf16 [M, 64]."""
    (W1, b1), (W2, b2), (W3, b3) = layers
    if isinstance(wts, ArenaRows):  # the dense features straight from the request arena
        if wts.arena.is_cuda:
            return hip().bottom_mlp3_arena(wts.arena, int(wts.B), int(nd), W1, b1, W2, b2, W3, b3)
        wts = _arena_unpack_host(wts)[1]
    if wts.is_cuda:
        return hip().bottom_mlp3(_rows(wts), int(nd), W1, b1, W2, b2, W3, b3)
    x = torch.zeros(wts.shape[0], W1.shape[1], dtype=torch.bfloat16)
    x[:, :nd] = wts[:, :nd].to(torch.bfloat16)
    for W, b in layers:
        x = linear(x, W, b, "relu")
    return x


# ------------------------------------------------------------------ K1b routing
def shard_route(ids, W: int, tm: int, col: torch.Tensor, mod: torch.Tensor, off: torch.Tensor,
                out: Optional[torch.Tensor] = None, hot: int = 1, wts: Optional[torch.Tensor] = None,
                out_w: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Embedding-parallel routing: int32 [W, B, tm * hot] with
    out[s, b, j * hot + h] = off[s*tm + j] + (ids[b, col[s*tm + j] + h] mod mod[s*tm + j]),
    i.e. the local row on owner rank s of its j-th table for candidate b (a
    multi-hot table's ``hot`` ids are consecutive columns); ``out_w`` gets the
    matching weights (multi-hot bags). ``ids`` may be :class:`ArenaRows`: the
    GPU kernel then reads ids and weights from the request bytes."""
    if isinstance(ids, ArenaRows):
        if ids.arena.is_cuda:
            return hip().shard_route(None, ids.arena, int(ids.B), int(ids.F), int(W), int(tm), col, mod, off, out,
                                     int(hot), None, out_w)
        ids, wts = _arena_unpack_host(ids)
    B, F = ids.shape
    if ids.is_cuda:
        return hip().shard_route(_rows(ids), None, int(B), int(F), int(W), int(tm), col, mod, off, out, int(hot),
                                 None if wts is None else _rows(wts), out_w)
    h = torch.arange(hot, dtype=torch.int64)
    c = (col.long().view(-1, 1) + h.view(1, -1)).clamp(0, F - 1).view(-1)  # [W*tm*hot]
    md = mod.view(-1, 1).expand(-1, hot).reshape(-1)
    of = off.view(-1, 1).expand(-1, hot).reshape(-1)
    r = (of.view(1, -1) + torch.remainder(ids.long()[:, c], md.view(1, -1))).to(torch.int32)  # [B, W*tm*hot]
    r = r.view(B, W, tm * hot).transpose(0, 1).contiguous()
    if out_w is not None:
        w = (wts.float()[:, c] if wts is not None else torch.ones(B, c.numel())).view(B, W, tm * hot)
        out_w.copy_(w.transpose(0, 1).reshape(out_w.shape))
    if out is not None:
        out.copy_(r.view(out.shape))
        return out
    return r


# ------------------------------------------------------------------ K6
def _extra_logit(extra: torch.Tensor, M: int) -> torch.Tensor:
    """A head's extra logit: fp32 [M], or [P, >= M] partial logits summed in
    row order (embed_gemm's first-order + FM partitions)."""
    if extra.dim() == 2:
        return extra[:, :M].float().sum(0)
    return extra.float()


def head(x: torch.Tensor, w: torch.Tensor, bias: float = 0.0, extra: Optional[torch.Tensor] = None,
         sigmoid: bool = True) -> torch.Tensor:
    """CTR head: act(x . w + bias + extra) -> fp32 [M] (``extra``: see _extra_logit)."""
    if x.is_cuda:
        return hip().head(x.contiguous(), w, float(bias), extra, sigmoid)
    y = x.float() @ w.float() + float(bias)
    if extra is not None:
        y = y + _extra_logit(extra, y.shape[0])
    return torch.sigmoid(y) if sigmoid else y


def linear_head_ok(x: torch.Tensor, W: torch.Tensor) -> bool:
    """Shapes the fused last-layer+head kernel covers (bf16, K % 64, N <= 256)."""
    return (x.dtype == torch.bfloat16 and W.dtype == torch.bfloat16 and x.shape[1] % 64 == 0
            and 0 < W.shape[0] <= 256)


def linear_head(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, act: str, hw: torch.Tensor, hbias: float = 0.0,
                extra: Optional[torch.Tensor] = None, sigmoid: bool = True,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K4+K6 fused: out_act(act(x W^T + b) . hw + hbias + extra) -> fp32 [M].

    The [M, N] activation of the last MLP layer never leaves registers; ``out``
    may be pinned host memory (the kernel then writes scores to the host)."""
    if x.is_cuda:
        return hip().gemm_head(x.contiguous(), W, b, _ACTS[act], hw, float(hbias), extra, sigmoid, out)
    h = x.float() @ W.float().t() + b.float()
    if act == "relu":
        h = torch.relu(h)
    y = h @ hw.float() + float(hbias)  # the fused kernel keeps h in fp32 (no bf16 round trip)
    if extra is not None:
        y = y + _extra_logit(extra, y.shape[0])
    y = torch.sigmoid(y) if sigmoid else y
    if out is not None:
        out.copy_(y)
        return out
    return y


def pack_bfrag(W: torch.Tensor) -> torch.Tensor:
    """bf16 weights [N, K] -> MFMA B-fragment order (csrc/kernels/mlp_tail.hip):
    block (n16, k64, kk) is 64 lanes x 8 values, lane (fr, fq) holding
    W[16 n16 + fr, 64 k64 + 32 kk + 8 fq + e] - one wave-instruction per
    fragment reads 1 KiB of contiguous bytes."""
    N, K = W.shape
    if N % 16 or K % 64:
        raise ValueError(f"pack_bfrag needs N % 16 == 0 and K % 64 == 0, got {tuple(W.shape)}")
    return W.reshape(N // 16, 16, K // 64, 2, 4, 8).permute(0, 2, 3, 4, 1, 5).contiguous()


def pack_frag32(W: torch.Tensor) -> torch.Tensor:
    """bf16 weights [N, K] -> the A-operand fragment order of
    v_mfma_f32_32x32x16_bf16 (csrc/kernels/gather_gemm.hip): block (n32, k64,
    s) is 64 lanes x 8 values, lane (r, h) = (l & 31, l >> 5) holding
    W[32 n32 + r, 64 k64 + 16 s + 8 h + e] - 1 KiB contiguous per fragment."""
    N, K = W.shape
    if N % 32 or K % 64:
        raise ValueError(f"pack_frag32 needs N % 32 == 0 and K % 64 == 0, got {tuple(W.shape)}")
    return W.reshape(N // 32, 32, K // 64, 4, 2, 8).permute(0, 2, 3, 4, 1, 5).contiguous()


# The fused MLP tail replaces GEMM2 + the fused last-layer/head kernel at or
# above this many rows (one 64-row workgroup per CU at 16384).
MLP_TAIL_MIN_ROWS = 8192


def mlp_tail_ok(x: torch.Tensor, l2, l3) -> bool:
    """Shapes the fused two-layer tail + head kernel covers: bf16 [M, 1024] ->
    512 -> 256 -> score, ReLU / linear layers, enough rows to fill the GPU."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1
            and x.shape[1] == 1024 and x.shape[0] >= MLP_TAIL_MIN_ROWS
            and not l2.fp8 and not l3.fp8 and tuple(l2.weight.shape) == (512, 1024)
            and tuple(l3.weight.shape) == (256, 512) and l2.act in ("relu", "none") and l3.act in ("relu", "none"))


def mlp_tail(x: torch.Tensor, W2p: torch.Tensor, b2: torch.Tensor, act2: str, W3p: torch.Tensor,
             b3: torch.Tensor, act3: str, hw: torch.Tensor, hbias: float = 0.0,
             extra: Optional[torch.Tensor] = None, sigmoid: bool = True,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K4 + K4 + K6 fused (GPU): out_act(act3(bf16(act2(x W2^T + b2)) W3^T + b3) . hw + hbias + extra).
    ``W2p`` / ``W3p``: :func:`pack_bfrag` of the two weights. ``out`` may be
    pinned host memory (the kernel writes the scores there)."""
    return hip().mlp_tail(x, W2p, b2, _ACTS[act2], W3p, b3, _ACTS[act3], hw, float(hbias), extra, sigmoid, out)


# The whole DeepFM / Wide&Deep tower as one kernel (gather_mlp.hip) at or above
# this many rows (16384 rows = one 64-row workgroup per CU).
GATHER_MLP_MIN_ROWS = 8192


def gather_mlp_ok(table: torch.Tensor, layers, rows: int) -> bool:
    """Shapes the one-launch tower covers: bf16 64-wide table of <= 2^25 rows,
    bf16 layers 64F -> 1024 (ReLU) -> 512 -> 256, enough rows to fill the GPU."""
    if len(layers) != 3 or rows < GATHER_MLP_MIN_ROWS:
        return False
    l1, l2, l3 = layers
    return (table.is_cuda and table.dtype == torch.bfloat16 and table.dim() == 2 and table.shape[1] == 64
            and table.shape[0] <= 2 ** 25 and not any(l.fp8 for l in layers)
            and tuple(l1.weight.shape) == (1024, l1.in_dim) and l1.k == l1.in_dim and l1.in_dim % 64 == 0
            and 1 <= l1.in_dim // 64 <= 64 and tuple(l2.weight.shape) == (512, 1024)
            and tuple(l3.weight.shape) == (256, 512) and l1.act == "relu" and l2.act in ("relu", "none")
            and l3.act in ("relu", "none"))


def gather_mlp(table: torch.Tensor, ids, wts: Optional[torch.Tensor], lin: Optional[torch.Tensor], modulo: int,
               bias: float, layers, hw: torch.Tensor, hbias: float, fm: bool, sigmoid: bool = True,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """K0 + K1 + K2 + K4 x 3 + K6 in one launch (GPU): the scores of a
    DeepFM (``fm``) or Wide&Deep tower, out_act(mlp(x) . hw + hbias + bias +
    sum_f lin[row] w (+ FM)), x[b, 64f:64f+64] = bf16(T[row(b, f)] * w(b, f)).
    Each workgroup resolves its own rows' ids / weights into LDS; h1 and h2
    stay in the CU's LDS (csrc/kernels/gather_mlp.hip). ``ids`` may be
    :class:`ArenaRows` (the request bytes); ``out``: device or pinned host scores."""
    l1, l2, l3 = layers
    m = int(modulo) if modulo > 0 else table.shape[0]
    args = (l1.packed("32"), l1.bias, l2.packed("32"), l2.bias, _ACTS[l2.act], l3.packed("32"), l3.bias,
            _ACTS[l3.act], hw, float(hbias), bool(fm), bool(sigmoid), out)
    if isinstance(ids, ArenaRows):
        return hip().gather_mlp(table, lin, ids.arena, None, None, int(ids.B), int(ids.F), m, float(bias), *args)
    return hip().gather_mlp(table, lin, None, _rows(ids), None if wts is None else _rows(wts), int(ids.shape[0]),
                            int(ids.shape[1]), m, float(bias), *args)


def unpack_bfrag(Wp: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """Inverse of :func:`pack_bfrag` (tests)."""
    return Wp.reshape(N // 16, K // 64, 2, 4, 16, 8).permute(0, 4, 1, 2, 3, 5).reshape(N, K)


# ------------------------------------------------------------------ K7
def sort_scores(scores: torch.Tensor, descending: bool = False, k: int = -1):
    """Sorted scores + the candidate permutation (the reference drops the latter,
    DCNClient.java:195). GPU: bitonic sort in LDS up to 8192 scores."""
    n = scores.numel()
    if k < 0 or k > n:
        k = n
    if scores.is_cuda and n <= hip().sort_max_elems():
        s, p = hip().sort_scores(scores.contiguous().float(), descending, int(k))
        return s, p
    if scores.is_cuda:  # large lists: library sort (plain, not a hot fused op)
        s, p = torch.sort(scores.float(), descending=descending, stable=True)
        return s[:k], p[:k]
    s, p = torch.sort(scores.float(), descending=descending, stable=True)
    return s[:k], p[:k]

"""Parameter containers shared by the CTR model families.

Weights are stored the way the kernels read them: embedding tables bf16
[rows, D], dense weights bf16 [out, in] (reduction dim contiguous), biases and
small vectors fp32. fp8 towers keep an OCP e4m3 copy of each weight with a
per-output-channel fp32 scale.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
from torch import nn

from .. import ops

DTYPES = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


def pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def make_generator(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def init_uniform_(t: torch.Tensor, bound: float, gen: torch.Generator) -> torch.Tensor:
    with torch.no_grad():
        if t.dtype in (torch.float32, torch.float64):
            t.uniform_(-bound, bound, generator=gen)
        else:  # draw in fp32 chunks to keep bf16 init device-side and bounded in memory
            flat = t.view(-1)
            step = 1 << 26
            for i in range(0, flat.numel(), step):
                n = min(step, flat.numel() - i)
                buf = torch.empty(n, dtype=torch.float32, device=t.device).uniform_(-bound, bound, generator=gen)
                flat[i:i + n].copy_(buf)
    return t


_M64 = (1 << 64) - 1


def _s64(c: int) -> int:
    """uint64 constant -> the int64 with the same bits (torch has no uint64 math)."""
    return c - (1 << 64) if c >= (1 << 63) else c


def _lsr(z: torch.Tensor, s: int) -> torch.Tensor:
    """Logical right shift of int64 bits."""
    return torch.bitwise_and(torch.bitwise_right_shift(z, s), (1 << (64 - s)) - 1)


def hashed_rows_at(rows: torch.Tensor, D: int, table_id: int, seed: int, bound: float) -> torch.Tensor:
    """The values hashed_uniform_rows_ gives table ``table_id``'s rows ``rows``
    (int64, any order / repeats) -> fp32 [len(rows), D]: an fp32 reference can
    rebuild just the rows a request touches (bench.py's sparse check)."""
    dev = rows.device
    cols = torch.arange(D, device=dev, dtype=torch.int64)
    salt = _s64((seed * 0x9E3779B97F4A7C15 + table_id * 0xD1B54A32D192ED03) & _M64)
    z = rows.to(torch.int64).view(-1)[:, None] * D + cols[None, :] + salt
    z = z + _s64(0x9E3779B97F4A7C15)
    z = torch.bitwise_xor(z, _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = torch.bitwise_xor(z, _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    z = torch.bitwise_xor(z, _lsr(z, 31))
    u = _lsr(z, 40).to(torch.float32) * (1.0 / (1 << 24))  # top 24 bits -> [0, 1)
    return (u * 2.0 - 1.0) * bound


def hashed_uniform_rows_(out: torch.Tensor, table_id: int, row_lo: int, seed: int, bound: float,
                         chunk_rows: int = 1 << 19) -> torch.Tensor:
    """Fill ``out`` [n, D] with U(-bound, bound) values that depend only on
    (seed, table_id, global row, column): any row shard of a table can be
    initialised on its own rank, and a sharded model matches the unsharded one
    bit for bit (splitmix64 of the element index; identical on CPU and GPU)."""
    n, D = out.shape
    dev = out.device
    with torch.no_grad():
        for r0 in range(0, n, chunk_rows):
            r1 = min(n, r0 + chunk_rows)
            rows = torch.arange(row_lo + r0, row_lo + r1, device=dev, dtype=torch.int64)
            out[r0:r1].copy_(hashed_rows_at(rows, D, table_id, seed, bound))
    return out


class Dense(nn.Module):
    """One fully connected layer: y = act(x W^T + b) (K4 MFMA GEMM)."""

    def __init__(self, in_dim: int, out_dim: int, act: str, dtype, device, gen, in_pad: Optional[int] = None,
                 fp8: bool = False):
        super().__init__()
        self.in_dim, self.out_dim, self.act = in_dim, out_dim, act
        self.k = in_pad if in_pad is not None else pad8(in_dim)
        bound = math.sqrt(6.0 / (in_dim + out_dim)) * (math.sqrt(2.0) if act == "relu" else 1.0)
        w = torch.zeros(out_dim, self.k, dtype=dtype, device=device)  # K padded to 16-byte rows
        w[:, :in_dim].copy_(init_uniform_(torch.empty(out_dim, in_dim, device=device), bound, gen))
        self.weight = nn.Parameter(w, requires_grad=False)
        self.bias = nn.Parameter(init_uniform_(torch.empty(out_dim, dtype=torch.float32, device=device), 0.01, gen),
                                 requires_grad=False)
        self.fp8 = fp8
        if fp8:
            self.quantize_fp8()

    def quantize_fp8(self) -> None:
        wf = self.weight.float()
        amax = wf.abs().amax(dim=1)
        sw = torch.where(amax > 0, amax / ops.FP8_MAX, torch.ones_like(amax))
        q = (wf / sw[:, None]).clamp(-ops.FP8_MAX, ops.FP8_MAX).to(torch.float8_e4m3fn)
        kq = -(-q.shape[1] // ops.FP8_K_PAD) * ops.FP8_K_PAD  # zero K padding: whole 128-deep MFMA tiles
        if kq != q.shape[1]:
            q = torch.cat([q, torch.zeros(q.shape[0], kq - q.shape[1], dtype=q.dtype, device=q.device)], dim=1)
        self.register_buffer("w_fp8", q.contiguous(), persistent=False)
        self.register_buffer("w_scale", sw.contiguous(), persistent=False)
        self.fp8 = True

    def packed(self, layout: str = "16") -> torch.Tensor:
        """The weight in MFMA fragment order - "16": ops.pack_bfrag (the fused
        MLP tail's 16x16x32 B operand), "32": ops.pack_frag32 (the gather-GEMM's
        and the one-launch tower's 32x32x16 A operand) - re-packed whenever the weight changed
        (load_state_dict bumps its version). Built by the eager warm-up that
        precedes every graph capture."""
        key = (self.weight.data_ptr(), self.weight._version)
        cache = self.__dict__.setdefault("_packed", {})
        cached = cache.get(layout)
        if cached is None or cached[0] != key:
            w = self.weight.detach()
            fresh = ops.pack_bfrag(w) if layout == "16" else ops.pack_frag32(w)
            if cached is not None and cached[1].shape == fresh.shape and cached[1].dtype == fresh.dtype:
                # a weight changed in place: re-pack INTO the buffer captured HIP
                # graphs already read (a new allocation would leave them serving
                # the old weights)
                cached[1].copy_(fresh)
                fresh = cached[1]
            cached = (key, fresh)
            cache[layout] = cached
        return cached[1]

    def forward(self, x: torch.Tensor, xq=None) -> torch.Tensor:
        """``xq``: (q, scale) of x already quantised by the caller (fp8 layers)."""
        if self.fp8:
            xq, sx = xq if xq is not None else ops.quant_rows_fp8(x, ops.FP8_K_PAD)
            return ops.linear_fp8(xq, sx, self.w_fp8, self.w_scale, self.bias, self.act)
        return ops.linear(x, self.weight, self.bias, self.act)


class MLP(nn.Module):
    def __init__(self, in_dim: int, dims: Sequence[int], dtype, device, gen, fp8: bool = False,
                 last_act: str = "relu", in_pad: Optional[int] = None):
        """``in_pad``: the first layer's K (>= in_dim, zero weight columns)."""
        super().__init__()
        layers: List[Dense] = []
        d = in_dim
        for i, h in enumerate(dims):
            act = "relu" if i < len(dims) - 1 else last_act
            layers.append(Dense(d, h, act, dtype, device, gen, fp8=fp8, in_pad=in_pad if i == 0 else None))
            d = h
        self.layers = nn.ModuleList(layers)
        self.out_dim = d

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        for layer in self.layers:
            x = layer(x)
        return x

    def forward_head(self, x: torch.Tensor, head_w: torch.Tensor, head_b: float,
                     extra: Optional[torch.Tensor] = None, sigmoid: bool = True,
                     out: Optional[torch.Tensor] = None, xq=None, start: int = 0) -> torch.Tensor:
        """MLP then CTR head. On the GPU the last layer and the head run as one
        kernel (ops.linear_head) whenever its shape allows; it writes ``out``
        (device or pinned host memory) directly. When exactly two layers remain
        (1024 -> 512 -> 256) on a batch that fills the GPU, both layers and the
        head run as ONE kernel (ops.mlp_tail: 64-row workgroups, h2 kept in LDS,
        weights loaded in MFMA fragment order straight into registers).
        ``start``: x is already the output of layers[:start]."""
        n = len(self.layers)
        k = start
        while n - k > 2:  # the layers in front of the tail (DCN-v2: the fp8 first layer)
            x = self.layers[k](x, xq if k == start else None)
            k += 1
        if n - k == 2 and x.is_cuda and (xq is None or k > start) and ops.mlp_tail_ok(x, *self.layers[k:]):
            l2, l3 = self.layers[k:]
            return ops.mlp_tail(x, l2.packed(), l2.bias, l2.act, l3.packed(), l3.bias, l3.act, head_w, head_b,
                                extra=extra, sigmoid=sigmoid, out=out)
        for j in range(k, n - 1):
            x = self.layers[j](x, xq if j == start else None)
        last = self.layers[-1]
        if x.is_cuda and not last.fp8 and last.act in ("relu", "none") and ops.linear_head_ok(x, last.weight):
            return ops.linear_head(x, last.weight, last.bias, last.act, head_w, head_b, extra=extra, sigmoid=sigmoid,
                                   out=out)
        y = ops.head(last(x), head_w, head_b, extra=extra, sigmoid=sigmoid)
        if out is not None:
            out.copy_(y, non_blocking=True)
            return out
        return y

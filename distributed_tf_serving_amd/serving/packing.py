"""Packed request rows: the one buffer a batch lives in from decode to kernel.

A candidate row is laid out as::

    [ feat_ids: F x int64 | feat_wts: F x fp32 | pad to 8 bytes ]

so a whole batch is ONE [rows, W] int64 tensor (W = row bytes / 8). The native
decoder writes PredictRequest payloads straight into a pinned host buffer of
this layout, one H2D copy moves it, one RCCL all-to-all fans it out across
GPUs, and the embedding kernel reads ids and weights in place through strided
row views (no unpacking pass). Ids travel as raw int64: hashing onto table rows
(K0) happens inside the gather kernel on the GPU, not on the host.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass(frozen=True)
class PackedLayout:
    fields: int

    @property
    def row_bytes(self) -> int:
        b = 12 * self.fields
        return b + (b % 8)

    @property
    def words(self) -> int:
        return self.row_bytes // 8

    def alloc(self, rows: int, device="cpu", pin: bool = False) -> torch.Tensor:
        t = torch.zeros((rows, self.words), dtype=torch.int64, device=device, pin_memory=pin)
        return t

    def ids(self, buf: torch.Tensor) -> torch.Tensor:
        """int64 [rows, F] row view."""
        return buf[:, : self.fields]

    def wts(self, buf: torch.Tensor) -> torch.Tensor:
        """fp32 [rows, F] row view."""
        return buf.view(torch.float32)[:, 2 * self.fields: 3 * self.fields]

    def pack(self, ids: torch.Tensor, wts: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        rows = ids.shape[0]
        buf = self.alloc(rows, device=ids.device) if out is None else out
        self.ids(buf)[:rows].copy_(ids)
        self.wts(buf)[:rows].copy_(wts)
        return buf

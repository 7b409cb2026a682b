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
    """``narrow_modulo`` > 0: the narrow row [int32 table rows x F | fp32
    weights x F] - ids already hashed (id mod m, the model's table size), 8
    bytes per field instead of 12. The candidate fan-out exchanges rows in
    this form (2/3 of the xGMI bytes); the gather reads
    int32 rows and fp32 weights in place. Weights stay fp32 (not bf16): a
    request's scores must not depend on its wire encoding or on the path it
    took through the server."""

    fields: int
    narrow_modulo: int = 0

    @property
    def narrow(self) -> bool:
        return self.narrow_modulo > 0

    @property
    def row_bytes(self) -> int:
        b = (8 if self.narrow else 12) * self.fields
        return (b + 7) // 8 * 8

    @property
    def words(self) -> int:
        return self.row_bytes // 8

    def alloc(self, rows: int, device="cpu", pin: bool = False) -> torch.Tensor:
        t = torch.zeros((rows, self.words), dtype=torch.int64, device=device, pin_memory=pin)
        return t

    def ids(self, buf: torch.Tensor) -> torch.Tensor:
        """int64 [rows, F] row view (narrow: int32 table rows)."""
        if self.narrow:
            return buf.view(torch.int32)[:, : self.fields]
        return buf[:, : self.fields]

    def wts(self, buf: torch.Tensor) -> torch.Tensor:
        """fp32 [rows, F] row view."""
        if self.narrow:
            return buf.view(torch.float32)[:, self.fields: 2 * self.fields]
        return buf.view(torch.float32)[:, 2 * self.fields: 3 * self.fields]

    def pack(self, ids: torch.Tensor, wts: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
        rows = ids.shape[0]
        buf = self.alloc(rows, device=ids.device) if out is None else out
        if self.narrow:
            ids = torch.remainder(ids.long(), self.narrow_modulo).to(torch.int32)
        self.ids(buf)[:rows].copy_(ids)
        self.wts(buf)[:rows].copy_(wts)
        return buf


# families whose forward hashes every id with ONE modulo (cfg.vocab_size) and
# reads ids / weights only in the embedding gather
NARROW_FAMILIES = ("wdl", "deepfm", "dcn", "dcn_v2")


def host_narrow_modulo(cfg) -> int:
    """The modulo the host may apply to every id of a request before the GPU
    sees it (int32 rows on the wire), 0 if none: the single table of the
    shared-table families; for DLRM the per-table row count, which every
    table shares (its per-table offset is added on the GPU, so a 100M-row x
    30 table model still fits int32 rows; re-hashing a reduced row with the
    same modulo is the identity)."""
    if cfg.family in NARROW_FAMILIES:
        m = int(getattr(cfg, "vocab_size", 0))
    elif cfg.family == "dlrm":
        m = int(getattr(cfg, "table_rows", 0))
    else:
        m = 0
    return m if 0 < m < (1 << 31) else 0


def layout_for(cfg, fanout: bool) -> PackedLayout:
    """Packed rows a shard backend uses: narrow when the rows are exchanged
    between GPUs (candidate fan-out) and the model allows it."""
    narrow = fanout and cfg.family in NARROW_FAMILIES and 0 < int(getattr(cfg, "vocab_size", 0)) < (1 << 31)
    return PackedLayout(cfg.num_fields, int(cfg.vocab_size) if narrow else 0)

"""Request arena: the zero-copy ingest buffer (host pinned <-> device mirror).

Serialized PredictRequests sit in the arena's payload region (received there,
or copied in with :meth:`ArenaLayout.place`); the host parses only the protobuf
framing and writes one descriptor per request (:meth:`build`, native); one SDMA
copy moves descriptors + raw bytes to the GPU; the ``unpack_arena`` kernel
(csrc/kernels/ingest.hip) gathers packed candidate rows from them inside the
step's HIP graph. Requests that are not raw ``tensor_content`` int64/fp32 are
decoded on the host into arena scratch space in raw form, so the GPU side is
uniform.

Layout (shared with csrc): header (n_req int32 @0, total_rows int64 @8,
row_table_off int64 @16), descriptors {ids_off, wts_off, rows, dst_row} int64
@64, payload @ARENA_PAYLOAD_OFF; after the last request (and any scratch) a row
table {ids_off, wts_off} int32 per candidate row, so a GPU thread finds its
row's features with one load instead of a search over the descriptors.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import torch

from ..ops import native


@dataclass(frozen=True)
class ArenaLayout:
    fields: int
    max_rows: int
    max_requests: int = 1024
    # packed varint int64_val ids (the reference client's encoding) decoded on
    # the GPU (csrc/runtime/arena.h, csrc/kernels/ingest.hip) instead of on
    # the host pool: the H2D copy carries the compact wire bytes
    gpu_varint: bool = True

    @property
    def varint_chunks(self) -> int:
        """Chunk-table capacity handed to the host build (0: host decode)."""
        if not self.gpu_varint:
            return 0
        return native().arena_varint_capacity(self.max_rows, self.fields, self.max_requests)

    @property
    def varint_blocks(self) -> int:
        """Grid of the varint kernel (blocks loop over the chunks)."""
        return min(1024, self.varint_chunks)

    def decode_varints(self, arena_dev: torch.Tensor) -> None:
        """GPU varint decode of a built, copied arena (no-op grid if none)."""
        if self.gpu_varint:
            from ..ops import hip

            hip().arena_varint_decode(arena_dev, self.varint_blocks)

    @property
    def payload_off(self) -> int:
        return native().ARENA_PAYLOAD_OFF

    @property
    def capacity(self) -> int:
        # serialized rows (varints can reach ~14 B/feature) + host-decoded scratch (12 B/feature)
        # + the per-row offset table (8 B/row)
        per_row = 28 * self.fields + 8
        return (self.payload_off + self.max_rows * per_row + self.max_requests * 1024 + 128
                + 32 * self.varint_chunks)

    def alloc(self, device="cpu", pin: bool = False) -> torch.Tensor:
        return torch.zeros(self.capacity, dtype=torch.uint8, device=device, pin_memory=pin)

    def place(self, arena: torch.Tensor, requests: Sequence[bytes], start: int = 0) -> List[Tuple[int, int]]:
        """Copy serialized requests into the payload region; returns their spans."""
        return native().arena_place(arena, list(requests), start)

    def build(self, arena: torch.Tensor, spans: Sequence[Tuple[int, int]], ids_key="feat_ids", wts_key="feat_wts"):
        """Parse in place + write descriptors; returns ArenaBatch (rows/offsets/errors/used_bytes)."""
        return native().arena_build(arena, list(spans), ids_key, wts_key, self.fields, self.max_rows,
                                    self.varint_chunks)

    def unpack_cpu(self, arena: torch.Tensor, packed: torch.Tensor) -> torch.Tensor:
        native().arena_unpack_cpu(arena, packed, self.fields)
        return packed

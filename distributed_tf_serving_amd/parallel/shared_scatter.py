"""Bootstrap of the shared-arena scatter (csrc/runtime/shared_scatter.h).

Scatter mode is the reference topology: rank 0 is the only front door and
every request's candidates are split over the shards (reference
DCNClient.java:46-74 split, :146-164 dispatch + join). Over RCCL that means
rank 0's single PCIe link carries every rank's request bytes, then xGMI carries
them again. With the shared arena, rank 0's request arenas and score outputs
are one POSIX shared-memory segment that every rank of the node maps and
registers with its own GPU: per step each rank DMAs only its share of the
batch over its own link and writes its scores straight into rank 0's output
(no collective in the step). Same bootstrap as the step control
(parallel/control.py): rank 0 creates the segment under a random name,
publishes the name in the job's store, waits for every rank to attach and
unlinks the name.
"""
from __future__ import annotations

import datetime
import os
import secrets
import time

from .control import default_store


def create_shared_scatter(module, world: int, rank: int, fields: int, n_arenas: int, arena_cap: int, slots: int,
                          out_floats: int, store=None, prefix: str = "dtfs/scatter/0", node: int = -1,
                          register: bool = False, timeout_s: float = 60.0, expected_payload: int = 0):
    """A SharedScatter of ``module`` (``_hip`` for GPU ranks, which also
    register the mapping with their device, ``_native`` for CPU ranks).
    Not a collective: every rank calls it with the same ``prefix``.
    ``node``: this rank's NUMA node (-1 unknown). Every rank publishes its node;
    rank 0 places the segment on its own and, with ``expected_payload`` (bytes
    of a full batch), each rank's share of every arena on that rank's node
    (runtime/shared_scatter.h scatter_placement)."""
    store = store if store is not None else default_store()
    name_key, att_key = f"{prefix}/name", f"{prefix}/attached"
    store.set(f"{prefix}/node/{rank}", str(int(node)))
    if rank == 0:
        keys = [f"{prefix}/node/{r}" for r in range(world)]
        store.wait(keys, datetime.timedelta(seconds=timeout_s))
        rank_nodes = [int(store.get(k).decode()) for k in keys]
        name = f"/dtfs-sct-{os.getpid()}-{secrets.token_hex(6)}"
        seg = module.SharedScatter(name, world, 0, True, fields, n_arenas, arena_cap, slots, out_floats, node,
                                   rank_nodes if expected_payload > 0 else [], int(expected_payload))
        store.set(name_key, name)
    else:
        store.wait([name_key], datetime.timedelta(seconds=timeout_s))
        name = store.get(name_key).decode()
        seg = module.SharedScatter(name, world, rank, False)
    if register:
        seg.register_with_gpu()
    store.add(att_key, 1)
    if rank == 0:
        deadline = time.monotonic() + timeout_s
        try:
            while store.add(att_key, 0) < world:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"shared scatter {name}: only {store.add(att_key, 0)} of {world} ranks attached")
                time.sleep(0.002)
        finally:
            seg.unlink()
    return seg


def expected_row_bytes(fields: int, narrow_modulo: int = 0, narrow_wts_cols: int = 0) -> int:
    """Arena payload bytes one candidate row takes, for placing each rank's
    share of a batch on its NUMA node. Raw tensor_content: 8 B id + 4 B weight
    per feature + framing. Narrowed on the host (GPU live servers, the
    default; csrc/runtime/narrow.h): 3-byte rows for tables of <= 2^24 rows
    (else 4) + the row's weights + its 8-byte row-table entry. Weights are
    priced as fp32, the widest form a narrowed request carries (bf16-exact
    weights travel in 2 bytes, all-ones in none): the placement then matches
    the heaviest traffic, where it matters."""
    if narrow_modulo <= 0:
        return 12 * fields + 16
    idb = 3 if narrow_modulo <= (1 << 24) else 4
    wcols = narrow_wts_cols if 0 < narrow_wts_cols < fields else fields
    return idb * fields + 4 * wcols + 8


def live_narrowing(model, cuda: bool, narrow: bool = True):
    """(narrow_modulo, narrow_wts_cols) the live server will use for this model
    (serving/live.py: GPU servables narrow on the host by default)."""
    from ..serving.packing import host_narrow_modulo

    m = host_narrow_modulo(model.cfg) if (narrow and cuda) else 0
    wc = int(getattr(model, "narrow_weight_cols", lambda: 0)()) if m else 0
    return m, wc


def scatter_for_engine(ctx, fields: int, arena_cap: int, slots: int, max_rows_per_rank: int, tag: str = "serve",
                       store=None, n_arenas: int = 0, narrow_modulo: int = 0, narrow_wts_cols: int = 0):
    """The segment of a scatter-mode job on one node (None for one rank).
    ``n_arenas`` defaults to what the live server allocates (slots + 3).
    ``narrow_modulo`` / ``narrow_wts_cols``: the live server's host narrowing
    (serving/live.py), which sets how many bytes each rank's share takes."""
    if ctx.world <= 1:
        return None
    from ..ops import hip, native
    from ..utils.affinity import current_node

    cuda = ctx.device.type == "cuda"
    # a full batch's request bytes: where each rank's share of an arena will sit
    expected = ctx.world * max_rows_per_rank * expected_row_bytes(fields, narrow_modulo, narrow_wts_cols)
    return create_shared_scatter(hip() if cuda else native(), ctx.world, ctx.rank, fields, n_arenas or slots + 3,
                                 arena_cap, slots, ctx.world * max_rows_per_rank, store=store,
                                 prefix=f"dtfs/scatter/{tag}", node=current_node() if cuda else -1, register=cuda,
                                 expected_payload=expected)

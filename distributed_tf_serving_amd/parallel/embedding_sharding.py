"""Embedding model parallelism for DLRM-scale tables (BASELINE config 4).

The reference has ONE parallel axis: candidate data parallelism (it splits a
request's candidates across shard servers, reference DCNClient.java:46-74,
146-164), with a full model replica per shard. That cannot hold "100M-row
embedding tables": 30 sparse tables x 100M rows x 64 x bf16 = 384 GB, more
than one MI355X's 288 GB. This module adds the CTR analogue of expert
parallelism (collective C3):

* **Planner** (`plan_sharding`): places each table on one rank (table-wise,
  greedy largest-first onto the least-loaded rank) or splits it by row ranges
  over every rank (row-wise) when a table is too large for a balanced
  table-wise placement, and checks each rank's bytes against its HBM budget.
* **`ShardedEmbedding`**: the forward for one-hot sparse fields, with every
  rank holding only its shards.
  - table-wise: ids all-to-all (rank r sends the ids of the tables owned by s),
    a local gather over the owned tables for all ranks' rows (K1 kernel), then
    an embeddings all-to-all back;
  - row-wise: ids all-gather, a masked local gather (the K1 kernel zeroes ids
    outside the rank's row range), then a reduce-scatter (sum). Exactly one
    rank owns each row, so the bf16 sum is exact.
  Every message has a fixed shape for a given batch size (no count exchange),
  so the step stays HIP-graph capturable on RCCL.
  - peer (``ModelConfig.embedding_exchange = "peer"``, table-wise): no
    exchange at all - each rank maps its peers' stores (IPC) and the lookup
    loads every row where it lives over xGMI, hot remote rows from a per-rank
    replica cache refreshed from online counts (parallel/hot_cache.py); the
    bytes crossing xGMI are the cache misses x 128.
* **`ShardedDLRM`**: the DLRM forward with sharded tables; dense towers are
  replicated and run data-parallel over each rank's candidates.

xGMI sizing: each all-to-all moves B x T_owned x 64 x 2 bytes per peer, one
peer per xGMI link (7 links), so it is latency-bound below ~1 MB per peer and
link-bound above; the planner's table-wise default keeps one message per step
per direction instead of one per table.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import nn

from .. import ops as ops_k
from ..config import ModelConfig
from ..models.ctr import DLRM
from ..models.layers import DTYPES, hashed_uniform_rows_
from . import hot_cache
from . import step_program as sp
from .dist import DistContext, split_rows

GiB = 1 << 30
MI355X_HBM_BYTES = 288 * 10 ** 9


@dataclass(frozen=True)
class TableSpec:
    name: str
    rows: int
    dim: int
    elem_bytes: int = 2

    @property
    def bytes(self) -> int:
        return self.rows * self.dim * self.elem_bytes


@dataclass
class Placement:
    table: int                    # index into ShardingPlan.tables
    kind: str                     # "table" | "row"
    rank: int = -1                # owner (table-wise)
    ranges: List[Tuple[int, int]] = field(default_factory=list)  # per-rank (lo, n) (row-wise)


@dataclass
class ShardingPlan:
    tables: List[TableSpec]
    world: int
    placements: List[Placement]
    budget_bytes: int

    def rank_bytes(self) -> List[int]:
        load = [0] * self.world
        for p in self.placements:
            t = self.tables[p.table]
            if p.kind == "table":
                load[p.rank] += t.bytes
            else:
                for r, (_, n) in enumerate(p.ranges):
                    load[r] += n * t.dim * t.elem_bytes
        return load

    def table_wise(self, rank: int) -> List[int]:
        """Tables rank owns whole, in table order."""
        return [p.table for p in self.placements if p.kind == "table" and p.rank == rank]

    def row_wise(self) -> List[int]:
        return [p.table for p in self.placements if p.kind == "row"]

    def placement(self, t: int) -> Placement:
        return next(p for p in self.placements if p.table == t)

    def describe(self) -> str:
        load = self.rank_bytes()
        lines = [f"sharding plan: {len(self.tables)} tables over {self.world} ranks, budget "
                 f"{self.budget_bytes / GiB:.1f} GiB/rank"]
        for r in range(self.world):
            tw = self.table_wise(r)
            lines.append(f"  rank {r}: {load[r] / GiB:.2f} GiB, table-wise {tw}")
        rw = self.row_wise()
        if rw:
            lines.append(f"  row-wise over all ranks: {rw}")
        mean = sum(load) / max(1, self.world)
        lines.append(f"  imbalance max/mean = {max(load) / max(mean, 1):.3f}")
        return "\n".join(lines)


def plan_sharding(tables: Sequence[TableSpec], world: int, budget_bytes: int = int(0.8 * MI355X_HBM_BYTES),
                  policy: str = "auto", row_wise_fraction: float = 0.5) -> ShardingPlan:
    """Place tables on ranks.

    ``policy``: "table" (all table-wise), "row" (all row-wise) or "auto":
    tables larger than ``row_wise_fraction`` x the mean per-rank load go
    row-wise (they would unbalance a table-wise placement), the rest go
    table-wise, largest first onto the least-loaded rank (LPT). Raises
    MemoryError when a rank exceeds ``budget_bytes`` (default: 80 % of one
    MI355X's 288 GB, leaving room for activations and the batching queue)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    tables = list(tables)
    total = sum(t.bytes for t in tables)
    mean = total / world
    placements: List[Optional[Placement]] = [None] * len(tables)
    load = [0] * world
    order = sorted(range(len(tables)), key=lambda i: -tables[i].bytes)
    for i in order:
        t = tables[i]
        row = policy == "row" or (policy == "auto" and world > 1 and t.bytes > row_wise_fraction * mean)
        if policy not in ("auto", "row", "table"):
            raise ValueError(f"unknown sharding policy {policy!r}")
        if row and world > 1:
            ranges = [(s, n) for s, n in split_rows(t.rows, world)]
            placements[i] = Placement(i, "row", ranges=ranges)
            for r, (_, n) in enumerate(ranges):
                load[r] += n * t.dim * t.elem_bytes
        else:
            r = min(range(world), key=lambda k: (load[k], k))
            placements[i] = Placement(i, "table", rank=r)
            load[r] += t.bytes
    plan = ShardingPlan(tables, world, [p for p in placements if p is not None], int(budget_bytes))
    over = [(r, b) for r, b in enumerate(plan.rank_bytes()) if b > budget_bytes]
    if over:
        r, b = over[0]
        raise MemoryError(f"rank {r} needs {b / GiB:.1f} GiB of tables, over its {budget_bytes / GiB:.1f} GiB "
                          f"budget; use more ranks or row-wise sharding\n{plan.describe()}")
    return plan


def dlrm_tables(cfg: ModelConfig) -> List[TableSpec]:
    eb = torch.tensor([], dtype=DTYPES[cfg.param_dtype]).element_size()
    return [TableSpec(f"t{f}", cfg.table_rows, cfg.embed_dim, eb) for f in range(cfg.num_sparse)]


class ShardedEmbedding(nn.Module):
    """This rank's shards of a set of one-hot embedding tables + the exchange,
    as step-program ops (parallel/step_program.py).

    ``program(ids, B, bufs)`` returns the aux-lane ops of one step for a batch
    of B candidates whose table ids are columns ``col_base + t`` of ``ids``
    ([B, F] int64/int32 row view); every rank runs the SAME B (the engine hands
    every rank a full bucket). Afterwards table t of candidate b is row
    ``map_off[t] + b * map_stride[t]`` of ``bufs["emb_all"]`` ([N, D] bf16),
    which the DLRM interaction kernel reads in place:

    * table-wise: ``shard_route`` writes each candidate's row on the owner,
      grouped by owner ([W, B, tmax] int32, hashed on the sender so the owner
      gathers with no modulo) -> ids all-to-all -> the owner gathers its
      tables for every rank's candidates -> embeddings all-to-all back;
    * row-wise: the same route with W = 1 (global table rows) -> all-gather ->
      masked gather (rows outside this rank's range contribute zeros) ->
      bf16 reduce-scatter (sum): exactly one rank owns each row, so it is exact.
    Every message has a fixed shape for a given B (no count exchange), so the
    step is capturable and replayed by the native StepRunner."""

    def __init__(self, plan: ShardingPlan, ctx: DistContext, seed: int, bound: float, dtype=torch.bfloat16,
                 device="cpu", group=None, col_base: int = 0, hot: int = 1, exchange: str = "alltoall",
                 cache_rows: int = 0, cache_sample_every: int = 8):
        super().__init__()
        self.plan, self.ctx, self.group = plan, ctx, group
        self.world, self.rank = plan.world, ctx.rank if plan.world > 1 else 0
        if exchange not in ("alltoall", "peer"):
            raise ValueError(f"unknown embedding exchange {exchange!r}")
        self.exchange = exchange
        self.col_base = int(col_base)
        # multi-hot: table t's ids are columns col_base + t * hot .. + hot - 1,
        # pooled (weighted sum) on the owner by the K1b bag kernel
        self.hot = int(hot)
        if self.hot > 1 and plan.row_wise():
            raise NotImplementedError("multi-hot tables shard table-wise (plan them with policy='table')")
        dev = torch.device(device)
        T = len(plan.tables)
        self.T = T
        self.D = plan.tables[0].dim if T else 0
        if any(t.dim != self.D for t in plan.tables):
            raise ValueError("all sharded tables must share one embedding dim")
        # ---- table-wise: tables owned here, and every rank's owned list
        self.tw_by_rank = [plan.table_wise(r) for r in range(self.world)]
        self.tmax = max((len(x) for x in self.tw_by_rank), default=0)
        self.rw = plan.row_wise()
        self.tw_tables = [t for t in range(T) if t not in self.rw]
        # local storage per rank: [owned table-wise tables | row-wise shards], one buffer
        def layout(r):
            rows, offs, segs = 0, {}, []
            for t in self.tw_by_rank[r]:
                offs[t] = rows
                segs.append((t, 0, plan.tables[t].rows, rows))
                rows += plan.tables[t].rows
            for t in self.rw:
                s, n = plan.placement(t).ranges[r]
                offs[t] = rows
                segs.append((t, s, n, rows))
                rows += n
            return rows, offs, segs

        lay = [layout(r) for r in range(self.world)]
        self.rows_local, my_off, self.segments = lay[self.rank]  # segments: (table, global lo, rows, local offset)
        peer = exchange == "peer" and self.world > 1
        if peer and self.rw:
            raise ValueError("the peer exchange shards table-wise (plan the tables with policy='table')")
        shm_tag = None
        if peer and dev.type == "cpu":  # peers map this rank's store from a shared-memory file
            import uuid

            tok: list = [None] * self.world
            dist.all_gather_object(tok, uuid.uuid4().hex[:12], group=group)
            shm_tag = f"/dev/shm/dtfs_peer_{tok[0]}_{self.rank}"
        if peer:
            # chunks of 8 M rows, each its own allocation (GPU: its own IPC
            # object - a peer maps exactly that chunk)
            chunks = hot_cache.alloc_store(self.rows_local, dtype, dev, shm_tag)
        else:
            chunks = [torch.empty(max(1, self.rows_local), self.D, dtype=dtype, device=dev)]
        per = chunks[0].shape[0]
        for t, s, n, o in self.segments:  # each segment's rows, chunk by chunk
            r = o
            while r < o + n:
                c, i = divmod(r, per)
                k = min(o + n - r, chunks[c].shape[0] - i)
                hashed_uniform_rows_(chunks[c][i:i + k], t, s + (r - o), seed, bound)
                r += k
        self.store = nn.Parameter(chunks[0], requires_grad=False)
        # the other chunks (peer exchange with > 8 M local rows)
        self.store_chunks = nn.ParameterList([nn.Parameter(c, requires_grad=False) for c in chunks[1:]])
        # peer exchange: every rank's store mapped here, each table's rows read
        # where they live, hot remote rows from this rank's replica cache
        self.peer: Optional[hot_cache.PeerTables] = None
        self.cache: Optional[hot_cache.HotRowCache] = None
        if exchange == "peer":
            mine = [c.data for c in [self.store, *self.store_chunks]]
            stores = hot_cache.open_peer_stores(mine, group, shm_tag) if peer else [mine]
            if shm_tag is not None:
                os.unlink(shm_tag)  # every rank has it mapped (open_peer_stores ends in a barrier)
            owner = [next(r for r in range(self.world) if t in self.tw_by_rank[r]) for t in range(T)]
            self.peer = hot_cache.PeerTables(stores, owner, [lay[owner[t]][1][t] for t in range(T)],
                                             [plan.tables[t].rows for t in range(T)], self.rank,
                                             chunk_shift=hot_cache.CHUNK_SHIFT if peer else None)
            if peer and cache_rows != 0 and self.peer.remote_tables:  # < 0: sized from free HBM
                self.cache = hot_cache.HotRowCache(self.peer, cache_rows, sample_every=cache_sample_every)
        i64 = dict(dtype=torch.int64, device=dev)
        # table-wise route: slot (s, j) <- table tw_by_rank[s][j] (pad: column 0, row 0 of s)
        cols, mods, offs = [], [], []
        for s in range(self.world):
            for j in range(self.tmax):
                if j < len(self.tw_by_rank[s]):
                    t = self.tw_by_rank[s][j]
                    cols.append(self.col_base + t * self.hot)
                    mods.append(plan.tables[t].rows)
                    offs.append(lay[s][1][t])
                else:
                    cols.append(self.col_base)
                    mods.append(1)
                    offs.append(0)
        self.register_buffer("tw_col", torch.tensor(cols or [0], dtype=torch.int32, device=dev), persistent=False)
        self.register_buffer("tw_mod", torch.tensor(mods or [1], **i64), persistent=False)
        self.register_buffer("tw_off", torch.tensor(offs or [0], **i64), persistent=False)
        # row-wise: route to global table rows, then the masked gather of my range
        Tr = len(self.rw)
        self.register_buffer("rw_col", torch.tensor([self.col_base + t for t in self.rw] or [0], dtype=torch.int32,
                                                    device=dev), persistent=False)
        self.register_buffer("rw_mod", torch.tensor([plan.tables[t].rows for t in self.rw] or [1], **i64),
                             persistent=False)
        self.register_buffer("rw_zero", torch.zeros(max(1, Tr), **i64), persistent=False)
        self.register_buffer("rw_off", torch.tensor([my_off[t] for t in self.rw] or [0], **i64), persistent=False)
        self.register_buffer("rw_lo", torch.tensor([plan.placement(t).ranges[self.rank][0] for t in self.rw] or [0],
                                                   **i64), persistent=False)
        self.register_buffer("rw_n", torch.tensor([plan.placement(t).ranges[self.rank][1] for t in self.rw] or [0],
                                                  **i64), persistent=False)
        # where table t of (local candidate) b lands after the exchange, per bucket B
        self._maps: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}

    def release_peers(self) -> None:
        """Unmap the other ranks' stores (GPU: closes their IPC mappings now;
        CPU: drops the shared-memory views). The device is drained first so no
        kernel still reads them; the lookup cannot run afterwards."""
        p = self.peer
        if p is None or self.world == 1 or getattr(self, "peers_released", False):
            return
        if self.store.is_cuda:
            torch.cuda.synchronize(self.store.device)
        p.stores = [chunks if r == self.rank else [] for r, chunks in enumerate(p.stores)]
        self.peers_released = True

    def local_bytes(self) -> int:
        return sum(c.numel() * c.element_size() for c in [self.store, *self.store_chunks])

    # -- exchange buffers / table map ----------------------------------------
    def n_tw_rows(self, B: int) -> int:
        return self.world * B * self.tmax if self.tw_tables else 0

    def alloc(self, B: int) -> Dict[str, torch.Tensor]:
        """Static exchange buffers of one (bucket, slot). One rank: the
        exchange is the identity, so receive buffers alias the send buffers
        and the lookup writes straight into ``emb_all`` (no collectives)."""
        dev, W, tm, D, Tr, hot = self.store.device, self.world, self.tmax, self.D, len(self.rw), self.hot
        i32 = dict(dtype=torch.int32, device=dev)
        bf = dict(dtype=self.store.dtype, device=dev)
        nt = self.n_tw_rows(B)
        bufs = {"emb_all": torch.zeros(max(1, nt + B * Tr), D, **bf)}
        if self.tw_tables:
            bufs["send_ids"] = torch.zeros(W, B, tm * hot, **i32)
            bufs["recv_ids"] = bufs["send_ids"] if W == 1 else torch.zeros(W, B, tm * hot, **i32)
            bufs["emb_send"] = bufs["emb_all"][:nt].view(W * B, tm * D) if W == 1 else torch.zeros(W * B, tm * D, **bf)
            if hot > 1:
                bufs["send_w"] = torch.zeros(W, B, tm * hot, dtype=torch.float32, device=dev)
                bufs["recv_w"] = bufs["send_w"] if W == 1 else torch.zeros(W, B, tm * hot, dtype=torch.float32,
                                                                               device=dev)
                bufs["bag_off"] = torch.arange(0, W * B * tm * hot + 1, hot, dtype=torch.int64, device=dev)
        if Tr:
            bufs["rw_ids"] = torch.zeros(1, B, Tr, **i32)
            bufs["rw_all"] = torch.zeros(W, B, Tr, **i32)
            bufs["rw_part"] = torch.zeros(W * B, Tr * D, **bf)
        return bufs

    def exchange_bytes(self, B: int) -> int:
        """Bytes this rank sends to OTHER ranks per step (ids + weights out,
        embeddings back): what crosses xGMI. Peer exchange: the rows this
        rank loads from peers with no replica cache (every remote lookup);
        the cache's counters give the measured bytes (misses x 128)."""
        W, tm, D, Tr, hot = self.world, self.tmax, self.D, len(self.rw), self.hot
        if W == 1:
            return 0
        eb = self.store.element_size()
        if self.peer is not None:
            return B * self.peer.remote_tables * hot * D * eb
        n = 0
        if self.tw_tables:
            n += (W - 1) * B * tm * hot * (4 + (4 if hot > 1 else 0))  # ids (+ weights) to the owners
            n += (W - 1) * B * tm * D * eb                             # pooled rows back to the requesters
        if Tr:
            n += (W - 1) * B * Tr * 4 + (W - 1) * B * Tr * D * eb      # all-gather ids, reduce-scatter rows
        return n

    def table_map(self, B: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """(emb_off, emb_stride) int64 [T]: table t of candidate b is row
        off[t] + b * stride[t] of emb_all (all-to-all recv region: [owner][b][j];
        reduce-scatter region after it: [b][i])."""
        m = self._maps.get(B)
        if m is None:
            off, stride = [0] * self.T, [1] * self.T
            for s in range(self.world):
                for j, t in enumerate(self.tw_by_rank[s]):
                    off[t], stride[t] = s * B * self.tmax + j, self.tmax
            base = self.n_tw_rows(B)
            for i, t in enumerate(self.rw):
                off[t], stride[t] = base + i, len(self.rw)
            dev = self.store.device
            m = self._maps[B] = (torch.tensor(off, dtype=torch.int64, device=dev),
                                 torch.tensor(stride, dtype=torch.int64, device=dev))
        return m

    # -- one step's aux-lane ops -----------------------------------------------
    def program(self, ids, B: int, bufs: Dict[str, torch.Tensor], wts: Optional[torch.Tensor] = None) -> List[sp.Op]:
        """``ids``: [B, F] row view (+ ``wts`` for multi-hot bags), or
        :class:`ops.ArenaRows` - the route kernel then reads ids and weights
        straight from the request bytes (K0 fused into the routing)."""
        W, tm, D, Tr, hot = self.world, self.tmax, self.D, len(self.rw), self.hot
        ops: List[sp.Op] = []

        def route():
            if self.tw_tables:
                ops_k.shard_route(ids, W, tm, self.tw_col, self.tw_mod, self.tw_off, out=bufs["send_ids"], hot=hot,
                                  wts=wts, out_w=bufs.get("send_w"))
            if Tr:
                ops_k.shard_route(ids, 1, Tr, self.rw_col, self.rw_mod, self.rw_zero[:Tr], out=bufs["rw_ids"])

        def lookup():
            if self.tw_tables:  # rows arrive hashed and offset: the gather needs no modulo
                if hot == 1:
                    ops_k.embed(self.store, bufs["recv_ids"].view(W * B, tm), None, modulo=self.store.shape[0],
                                want_x=True, out_x=bufs["emb_send"])
                else:  # K1b: weighted bags of `hot` rows, pooled on the owner
                    ops_k.embedding_bag(self.store, bufs["recv_ids"].view(-1), bufs["bag_off"],
                                        per_sample_weights=bufs["recv_w"].view(-1), modulo=self.store.shape[0],
                                        out_bf16=True, out=bufs["emb_send"].view(W * B * tm, D))
            if Tr:
                ops_k.embed(self.store, bufs["rw_all"].view(W * B, Tr), None, modulo_f=self.rw_mod,
                            offset_f=self.rw_off, want_x=True, out_x=bufs["rw_part"], shard_lo_f=self.rw_lo,
                            shard_n_f=self.rw_n)

        ops.append(sp.Kernels(sp.AUX, route, "route"))
        ops.append(sp.Sync("record", sp.AUX, 0))  # ids routed: the dense tower may read the batch
        if self.tw_tables and W > 1:
            ops.append(sp.Coll("alltoall", sp.AUX, bufs["send_ids"], bufs["recv_ids"]))
            if hot > 1:
                ops.append(sp.Coll("alltoall", sp.AUX, bufs["send_w"], bufs["recv_w"]))
        if Tr:
            ops.append(sp.Coll("allgather", sp.AUX, bufs["rw_ids"], bufs["rw_all"]))
        ops.append(sp.Kernels(sp.AUX, lookup, "lookup"))
        nt = self.n_tw_rows(B)
        if self.tw_tables and W > 1:
            ops.append(sp.Coll("alltoall", sp.AUX, bufs["emb_send"], bufs["emb_all"][:nt]))
        if Tr:
            ops.append(sp.Coll("reduce_scatter", sp.AUX, bufs["rw_part"], bufs["emb_all"][nt:nt + B * Tr]))
        return ops

    def forward(self, ids: torch.Tensor, wts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Eager exchange (collective unless peer): ids [B, F] (tables at
        columns col_base..) -> [B, T, D]."""
        B = ids.shape[0]
        if self.peer is not None:
            w = wts.float() if wts is not None else torch.ones(ids.shape, dtype=torch.float32, device=ids.device)
            return ops_k.peer_bag(ids, w, B, self.col_base, self.hot, self.peer, self.cache)
        bufs = self.alloc(B)
        w = None if wts is None else wts.float().contiguous()
        sp.run_eager(self.program(ids.contiguous(), B, bufs, w), self.group)
        off, stride = self.table_map(B)
        rows = off.view(1, -1) + torch.arange(B, device=off.device).view(-1, 1) * stride.view(1, -1)
        return bufs["emb_all"][rows]


def peer_access_everywhere(ctx: DistContext, device: torch.device, group=None) -> bool:
    """True when this job's ranks are on GPUs that can all load from each
    other's memory (collective at world > 1): the peer exchange's condition.
    One rank, or the CPU: False (nothing to exchange / no peer mapping)."""
    world = ctx.world if ctx.is_distributed else 1
    if device.type != "cuda" or world == 1:
        return False
    mine = torch.cuda.current_device() if device.index is None else device.index
    devs: list = [None] * world
    dist.all_gather_object(devs, mine, group=group)
    ok = all(d == mine or torch.cuda.can_device_access_peer(mine, d) for d in devs)
    votes: list = [None] * world
    dist.all_gather_object(votes, bool(ok), group=group)
    return all(votes)


def build_parallel_model(cfg: ModelConfig, device, ctx: Optional[DistContext] = None, shard_tables: str = "auto",
                         policy: str = "auto", budget_bytes: int = int(0.8 * MI355X_HBM_BYTES), group=None):
    """The model a rank serves: DLRM tables are sharded across the process
    group when ``shard_tables`` is "on", or "auto" and the job has > 1 rank;
    every other family (and a 1-rank DLRM) is a full replica
    (candidate data parallelism, the reference's only axis)."""
    from ..models import build_model

    ctx = ctx or DistContext(device=torch.device(device))
    if cfg.family == "dlrm" and (shard_tables == "on" or (shard_tables == "auto" and ctx.is_distributed)):
        return ShardedDLRM(cfg, ctx, device=device, policy=policy, budget_bytes=budget_bytes, group=group).eval()
    return build_model(cfg, device)


class ShardedDLRM(nn.Module):
    """DLRM whose sparse tables are sharded across the process group.

    Dense towers (bottom / top MLP, head) are replicated - built from the same
    seed as ``models.ctr.DLRM`` so an unsharded DLRM gives identical scores -
    and run data-parallel on this rank's candidates. One step is a two-lane
    program (parallel/step_program.py): the table exchange on the aux lane,
    the bottom MLP overlapping it on the compute lane, then the interaction
    reads the exchanged embeddings in place and the top MLP + head finish."""

    family = "dlrm"

    def __init__(self, cfg: ModelConfig, ctx: DistContext, device="cpu", plan: Optional[ShardingPlan] = None,
                 policy: str = "auto", budget_bytes: int = int(0.8 * MI355X_HBM_BYTES), group=None):
        super().__init__()
        self.cfg, self.ctx, self.group = cfg, ctx, group
        self.hot = max(1, int(getattr(cfg, "multi_hot", 1)))
        world = ctx.world if ctx.is_distributed else 1
        exchange = getattr(cfg, "embedding_exchange", "alltoall")
        if exchange == "auto":
            exchange = "peer" if peer_access_everywhere(ctx, torch.device(device), group) else "alltoall"
        if (self.hot > 1 or exchange == "peer") and policy == "auto":
            # multi-hot bags pool on their table's owner; peers read whole
            # tables where they live
            policy = "table"
        self.plan = plan or plan_sharding(dlrm_tables(cfg), world, budget_bytes, policy)
        self.dense = DLRM(cfg, device=device, materialize_tables=False)
        self.dense.gen = None
        self.emb = ShardedEmbedding(self.plan, ctx, cfg.seed, self.dense.table_bound, DTYPES[cfg.param_dtype],
                                    device, group, col_base=cfg.num_dense, hot=self.hot, exchange=exchange,
                                    cache_rows=int(getattr(cfg, "hot_cache_rows", -1)))
        self.device_ = torch.device(device)

    def signature(self):
        return self.dense.signature()

    def param_bytes(self) -> int:
        return self.dense.param_bytes() + self.emb.local_bytes()

    def alloc(self, B: int) -> Dict[str, torch.Tensor]:
        if self._peer_step():
            e = self.emb
            return {"emb_all": torch.zeros(B * e.T, e.D, dtype=e.store.dtype, device=e.store.device)} if self.hot > 1 \
                else {}
        return self.emb.alloc(B)

    def _peer_step(self) -> bool:
        """The step reads every table where it lives (peer exchange, > 1 rank)."""
        return self.emb.peer is not None and self.emb.world > 1

    # -- hot-row replica cache (peer exchange) ---------------------------------
    @property
    def cache(self) -> Optional[hot_cache.HotRowCache]:
        return self.emb.cache

    def start_cache(self, interval_s: float = 1.0) -> None:
        """Refresh the replica cache from its online counts every interval_s."""
        if self.emb.cache is not None:
            self.emb.cache.start(interval_s)

    def stop_cache(self) -> None:
        if self.emb.cache is not None:
            self.emb.cache.stop()

    def release(self) -> None:
        """Shutdown, once no step can run any more (the live server drained):
        stop the replica-cache refresher and unmap every peer's store here, in
        program order, instead of from interpreter-teardown deleters racing a
        still-running refresher (the round-5 SIGABRT at cluster exit)."""
        self.stop_cache()
        self.emb.release_peers()

    def narrow_weight_cols(self) -> int:
        """One-hot: only the dense features' weights are read (the request
        arena carries just those, serving/live.py); multi-hot bags read all."""
        return self.cfg.num_dense if self.hot == 1 else 0

    @property
    def supports_arena(self) -> bool:
        """The step reads the request arena itself: the route kernel takes the
        sparse ids (and bag weights) from the request bytes, the fused bottom
        MLP the dense features - no unpack pass (parallel/fanout.py)."""
        return self.dense._bottom_fused() and self.dense.dtype == torch.bfloat16

    def exchange_bytes(self, B: int) -> int:
        return self.emb.exchange_bytes(B)

    def build_program(self, ids, wts: Optional[torch.Tensor], B: int, bufs: Dict[str, torch.Tensor],
                      out: Optional[torch.Tensor] = None, state: Optional[dict] = None) -> List[sp.Op]:
        """One step over static inputs: ids [B, F] / wts [B, F] row views, or
        ``ids`` = :class:`ops.ArenaRows` (wts None: both come from the request
        bytes); scores -> ``out`` (or ``state["scores"]``)."""
        d = self.dense
        st = {} if state is None else state
        arena = isinstance(ids, ops_k.ArenaRows)
        if self._peer_step():
            # peer exchange: no collective - the lookup loads each row from its
            # owner's HBM over xGMI (or this rank's replica cache), fused into
            # the interaction for one-hot tables, a pooled bag pass for multi-hot
            e, col0 = self.emb, self.cfg.num_dense
            bag_w = None if (arena or self.hot == 1) else (wts if wts.dtype == torch.float32 else wts.float())

            def peer_step():
                dense_out = d.bottom_out(ids if arena else (wts if wts.dtype == torch.float32 else wts.float()))
                if self.hot == 1:
                    z = ops_k.dot_interaction_gather_peer(dense_out, ids, e.peer, e.cache, d.inter_cols, id_col0=col0)
                else:
                    emb = ops_k.peer_bag(ids, bag_w, B, col0, self.hot, e.peer, e.cache,
                                         out=bufs["emb_all"].view(B, e.T, e.D))
                    z = ops_k.dot_interaction(dense_out, emb, d.inter_cols)
                st["scores"] = d.top.forward_head(z, d.head_w, d.head_b, out=out)

            return [sp.Sync("record", sp.AUX, 0), sp.Sync("wait", sp.COMPUTE, 0),
                    sp.Kernels(sp.COMPUTE, peer_step, "step")]
        fused = self._local_fused(ids)
        if fused is not None:
            # one rank, one-hot, table-wise: the exchange is the identity, so
            # the interaction kernel gathers the rows from this rank's store
            # itself, exactly like the unsharded DLRM (no route, no [B, T, 64]
            # round trip through HBM)
            mod, off = fused

            def step():
                dense_out = d.bottom_out(ids if arena else (wts if wts.dtype == torch.float32 else wts.float()))
                z = ops_k.dot_interaction_gather(dense_out, self.emb.store, ids if arena else d.sparse_ids(ids), mod,
                                                 off, d.inter_cols, id_col0=self.cfg.num_dense)
                st["scores"] = d.top.forward_head(z, d.head_w, d.head_b, out=out)

            return [sp.Sync("record", sp.AUX, 0), sp.Sync("wait", sp.COMPUTE, 0), sp.Kernels(sp.COMPUTE, step, "step")]
        emb_off, emb_stride = self.emb.table_map(B)
        bag_w = None
        if self.hot > 1 and not arena:
            bag_w = wts if wts.dtype == torch.float32 else wts.float()
        ops = self.emb.program(ids, B, bufs, bag_w)
        k = next(i for i, o in enumerate(ops) if isinstance(o, sp.Sync))  # after the route: the batch is read

        def bottom():
            if arena:  # the fused bottom tower reads the dense features from the arena
                st["dense"] = d.bottom_out(ids)
            else:
                w = wts if wts.dtype == torch.float32 else wts.float()
                st["dense"] = d.bottom_out(w)

        def top():
            z = ops_k.dot_interaction(st["dense"], bufs["emb_all"], d.inter_cols, emb_off, emb_stride)
            st["scores"] = d.top.forward_head(z, d.head_w, d.head_b, out=out)

        ops[k + 1:k + 1] = [sp.Sync("wait", sp.COMPUTE, 0), sp.Kernels(sp.COMPUTE, bottom, "bottom")]
        ops += [sp.Sync("record", sp.AUX, 1), sp.Sync("wait", sp.COMPUTE, 1), sp.Kernels(sp.COMPUTE, top, "top")]
        return ops

    def _local_fused(self, ids):
        """(modulo_f, offset_f) of every table in this rank's store when the
        whole lookup is local and fusable into the interaction (one rank,
        one-hot, table-wise, GPU), else None."""
        e = self.emb
        on_gpu = ids.arena.is_cuda if isinstance(ids, ops_k.ArenaRows) else ids.is_cuda
        if not (on_gpu and e.world == 1 and self.hot == 1 and not e.rw and e.T):
            return None
        if getattr(self, "_lf", None) is None:
            dev = e.store.device
            offs = dict((t, o) for t, _, _, o in e.segments)
            self._lf = (torch.tensor([t.rows for t in self.plan.tables], dtype=torch.int64, device=dev),
                        torch.tensor([offs[t] for t in range(e.T)], dtype=torch.int64, device=dev))
        return self._lf

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, wts: Optional[torch.Tensor], out: Optional[torch.Tensor] = None):
        """Eager step (collective: every rank calls it with the same B)."""
        B = ids.shape[0]
        st: dict = {}
        sp.run_eager(self.build_program(ids, wts, B, self.alloc(B), out=out, state=st), self.group)
        return st["scores"]

    @property
    def has_collectives(self) -> bool:
        """The forward issues collectives (every rank must run every step);
        the peer exchange has none: each rank's steps are its own."""
        return self.plan.world > 1 and not self._peer_step()

    supports_program = True

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
* **`ShardedDLRM`**: the DLRM forward with sharded tables; dense towers are
  replicated and run data-parallel over each rank's candidates.

xGMI sizing: each all-to-all moves B x T_owned x 64 x 2 bytes per peer, one
peer per xGMI link (7 links), so it is latency-bound below ~1 MB per peer and
link-bound above; the planner's table-wise default keeps one message per step
per direction instead of one per table.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import nn

from .. import ops
from ..config import ModelConfig
from ..models.ctr import DLRM
from ..models.layers import DTYPES, hashed_uniform_rows_
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


def _reduce_scatter_sum(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = this rank's slice (dim 0) of the sum over ranks of inp."""
    if dist.get_backend(group) == "gloo":  # gloo has no reduce_scatter; all-reduce in fp32 and slice
        full = inp.float()
        dist.all_reduce(full, group=group)
        r, n = dist.get_rank(group), out.shape[0]
        out.copy_(full[r * n:(r + 1) * n])
    else:
        dist.reduce_scatter_tensor(out, inp, group=group)


def _all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out[r*B:(r+1)*B] = rank r's inp."""
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.chunk(dist.get_world_size(group))), inp, group=group)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _coll_dtype(t: torch.Tensor, group) -> torch.Tensor:
    # gloo's CPU collectives: keep the wire dtype fp32 for bf16 payloads
    return t.float() if (t.dtype == torch.bfloat16 and dist.get_backend(group) == "gloo") else t


class ShardedEmbedding(nn.Module):
    """This rank's shards of a set of one-hot embedding tables + the exchange.

    ``forward(sparse_ids [B, T]) -> [B, T, D]`` on every rank with the SAME B
    (the fan-out engine hands every rank an equal slice)."""

    def __init__(self, plan: ShardingPlan, ctx: DistContext, seed: int, bound: float, dtype=torch.bfloat16,
                 device="cpu", group=None):
        super().__init__()
        self.plan, self.ctx, self.group = plan, ctx, group
        self.world, self.rank = plan.world, ctx.rank if plan.world > 1 else 0
        dev = torch.device(device)
        T = len(plan.tables)
        self.T = T
        self.D = plan.tables[0].dim if T else 0
        if any(t.dim != self.D for t in plan.tables):
            raise ValueError("all sharded tables must share one embedding dim")
        # ---- table-wise: tables owned here, and every rank's owned list
        self.tw_by_rank = [plan.table_wise(r) for r in range(self.world)]
        self.tmax = max((len(x) for x in self.tw_by_rank), default=0)
        mine = self.tw_by_rank[self.rank]
        self.rw = plan.row_wise()
        # local storage: [owned table-wise tables | row-wise shards], one buffer
        rows_local, mod, off, lo, nn_ = 0, [], [], [], []
        segs = []
        for t in mine:
            spec = plan.tables[t]
            segs.append((t, 0, spec.rows, rows_local))
            mod.append(spec.rows)
            off.append(rows_local)
            rows_local += spec.rows
        # pad the owned-table list to tmax with table 0 of this rank (lookups discarded)
        pad_mod = mod[0] if mod else 1
        while len(mod) < self.tmax:
            mod.append(pad_mod)
            off.append(0)
        rw_mod, rw_off, rw_lo, rw_n = [], [], [], []
        for t in self.rw:
            spec = plan.tables[t]
            s, n = plan.placement(t).ranges[self.rank]
            segs.append((t, s, n, rows_local))
            rw_mod.append(spec.rows)
            rw_off.append(rows_local)
            rw_lo.append(s)
            rw_n.append(n)
            rows_local += n
        self.rows_local = rows_local
        self.segments = segs  # (table, global row lo, rows, local offset)
        store = torch.empty(max(1, rows_local), self.D, dtype=dtype, device=dev)
        for t, s, n, o in segs:
            if n:
                hashed_uniform_rows_(store[o:o + n], t, s, seed, bound)
        self.store = nn.Parameter(store, requires_grad=False)
        i64 = dict(dtype=torch.int64, device=dev)
        self.register_buffer("tw_mod", torch.tensor(mod or [1], **i64), persistent=False)
        self.register_buffer("tw_off", torch.tensor(off or [0], **i64), persistent=False)
        self.register_buffer("rw_mod", torch.tensor(rw_mod or [1], **i64), persistent=False)
        self.register_buffer("rw_off", torch.tensor(rw_off or [0], **i64), persistent=False)
        self.register_buffer("rw_lo", torch.tensor(rw_lo or [0], **i64), persistent=False)
        self.register_buffer("rw_n", torch.tensor(rw_n or [0], **i64), persistent=False)
        # send-side column gather: slot (s, j) <- sparse column tw_by_rank[s][j] (pad: column 0)
        send_cols = []
        for s in range(self.world):
            cols = self.tw_by_rank[s] + [0] * (self.tmax - len(self.tw_by_rank[s]))
            send_cols += cols
        self.register_buffer("send_cols", torch.tensor(send_cols or [0], **i64), persistent=False)
        # receive-side: output table t <- flat slot owner(t) * tmax + j
        recv_slot = [0] * T
        for s in range(self.world):
            for j, t in enumerate(self.tw_by_rank[s]):
                recv_slot[t] = s * self.tmax + j
        self.register_buffer("recv_slot_tw", torch.tensor([recv_slot[t] for t in range(T) if t not in self.rw] or [0],
                                                          **i64), persistent=False)
        self.tw_tables = [t for t in range(T) if t not in self.rw]
        self.register_buffer("tw_cols", torch.tensor(self.tw_tables or [0], **i64), persistent=False)
        self.register_buffer("rw_cols", torch.tensor(self.rw or [0], **i64), persistent=False)

    def local_bytes(self) -> int:
        return self.store.numel() * self.store.element_size()

    # -- the exchange ------------------------------------------------------
    def _lookup(self, ids: torch.Tensor, mod, off, lo=None, n=None) -> torch.Tensor:
        x, _ = ops.embed(self.store, ids, None, modulo_f=mod, offset_f=off, want_x=True, shard_lo_f=lo, shard_n_f=n)
        return x

    def _table_wise(self, sparse: torch.Tensor) -> torch.Tensor:
        """-> [B, world * tmax, D]: slot s*tmax+j = table tw_by_rank[s][j] for my rows."""
        B, W, tm, D = sparse.shape[0], self.world, self.tmax, self.D
        send = sparse.index_select(1, self.send_cols).view(B, W, tm).transpose(0, 1).contiguous()  # [W, B, tm]
        if W > 1:
            recv = torch.empty_like(send)
            dist.all_to_all_single(recv, send, group=self.group)
        else:
            recv = send
        emb = self._lookup(recv.view(W * B, tm), self.tw_mod, self.tw_off).view(W, B, tm, D)  # my tables, all rows
        if W > 1:
            wire = _coll_dtype(emb, self.group)
            back = torch.empty_like(wire)
            dist.all_to_all_single(back, wire.contiguous(), group=self.group)
            back = back.to(emb.dtype)
        else:
            back = emb
        return back.permute(1, 0, 2, 3).reshape(B, W * tm, D)

    def _row_wise(self, sparse: torch.Tensor) -> torch.Tensor:
        """-> [B, T_rw, D]: partial lookups summed across ranks."""
        B, W, D = sparse.shape[0], self.world, self.D
        ids = sparse.index_select(1, self.rw_cols).contiguous()  # [B, T_rw]
        Tr = ids.shape[1]
        if W > 1:
            gathered = torch.empty(W * B, Tr, dtype=ids.dtype, device=ids.device)
            _all_gather_rows(gathered, ids, self.group)
        else:
            gathered = ids
        part = self._lookup(gathered, self.rw_mod, self.rw_off, self.rw_lo, self.rw_n)  # [W*B, Tr*D]
        if W > 1:
            wire = _coll_dtype(part, self.group)
            out = torch.empty(B, Tr * D, dtype=wire.dtype, device=wire.device)
            _reduce_scatter_sum(out, wire, self.group)
            part = out.to(part.dtype)
        return part.view(B, Tr, D)

    def forward(self, sparse_ids: torch.Tensor) -> torch.Tensor:
        B = sparse_ids.shape[0]
        sparse_ids = sparse_ids.contiguous()
        out = torch.empty(B, self.T, self.D, dtype=self.store.dtype, device=sparse_ids.device)
        if self.tw_tables:
            tw = self._table_wise(sparse_ids)
            out.index_copy_(1, self.tw_cols, tw.index_select(1, self.recv_slot_tw))
        if self.rw:
            out.index_copy_(1, self.rw_cols, self._row_wise(sparse_ids))
        return out


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
    and run data-parallel on this rank's candidates."""

    family = "dlrm"

    def __init__(self, cfg: ModelConfig, ctx: DistContext, device="cpu", plan: Optional[ShardingPlan] = None,
                 policy: str = "auto", budget_bytes: int = int(0.8 * MI355X_HBM_BYTES), group=None):
        super().__init__()
        self.cfg, self.ctx = cfg, ctx
        world = ctx.world if ctx.is_distributed else 1
        self.plan = plan or plan_sharding(dlrm_tables(cfg), world, budget_bytes, policy)
        self.dense = DLRM(cfg, device=device, materialize_tables=False)
        self.dense.gen = None
        self.emb = ShardedEmbedding(self.plan, ctx, cfg.seed, self.dense.table_bound, DTYPES[cfg.param_dtype],
                                    device, group)
        self.device_ = torch.device(device)

    def signature(self):
        return self.dense.signature()

    def param_bytes(self) -> int:
        return self.dense.param_bytes() + self.emb.local_bytes()

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, wts: Optional[torch.Tensor], out: Optional[torch.Tensor] = None):
        if wts is not None and wts.dtype != torch.float32:
            wts = wts.float()
        d = self.dense
        dense_out = d.bottom(d.dense_input(wts))
        emb = self.emb(d.sparse_ids(ids))
        return d.interact_and_top(dense_out, emb, out=out)

    @property
    def has_collectives(self) -> bool:
        """The forward issues collectives (not capturable into the step graph)."""
        return self.plan.world > 1

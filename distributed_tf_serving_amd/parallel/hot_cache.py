"""Peer lookup and the hot-row replica cache for table-wise sharded embeddings.

SURVEY §2.4 K1b / §2.5 C3 asks for embedding model parallelism over 8 GPUs;
the reference has no sharded embeddings at all (its TF-Serving shards each run
a full replica, reference ``README.md``). The exchange mode of
:class:`~.embedding_sharding.ShardedEmbedding` built here is MI355X-first:

* **Peer lookup** (``exchange="peer"``). The 8 GPUs of a node are fully
  connected by xGMI and every GPU can load from a peer's HBM. Each rank
  exports its table store once (IPC handle; on the CPU a shared-memory file),
  maps every peer's store, and the step's lookup kernel reads each candidate's
  row *where it lives*: no ids all-to-all, no lookup pass on the owner, no rows
  all-to-all, and no collective coupling the ranks' steps. The one-hot step is
  the same single fused kernel as one rank's (``dot_interact_gather_kernel``
  with the peer lookup on, csrc/kernels/interaction.hip); multi-hot bags pool
  through ``peer_bag_kernel`` (csrc/kernels/peer_lookup.hip).
* **Hot-row replica cache** (:class:`HotRowCache`). Most lookups of a skewed
  (Zipf) id stream hit a small set of rows. Each rank keeps copies of the hot
  rows of tables owned by OTHER ranks in HBM left over after its shard
  (288 GB per GPU), behind an open-addressing index; the lookup probes it
  first and goes over xGMI only on a miss, so the bytes crossing xGMI per step
  are ``misses x 128``. The hot set comes from online counts: the kernel pushes
  the remote keys of every ``sample_every``-th candidate into a ring, and
  :meth:`HotRowCache.refresh` (a background thread in serving, or called
  between steps) folds the ring into exponentially decayed counts, picks the
  top rows, copies the new ones from their owners into free slots and swaps
  in a freshly built index - never touching a slot or an index that a step in
  flight may read.

Keys are ``(t << 40) | row``. Counters: ``stats`` int64 [128] (hits at even,
misses at odd entries, summed by :meth:`HotRowCache.counts`).
"""
from __future__ import annotations

import os
import threading
import time
from contextlib import nullcontext
from typing import List, Optional, Sequence, Tuple

import torch

KEY_SHIFT = 40
ROW_MASK = (1 << KEY_SHIFT) - 1
D = 64


def _next_pow2(n: int) -> int:
    p = 2
    while p < n:
        p <<= 1
    return p


CHUNK_SHIFT = 23  # 8 M rows (1 GiB of bf16 rows) per store chunk


class PeerTables:
    """Where each table's rows live, seen from this rank. ``stores[r]`` is rank
    r's store as a list of chunks (chunk c = store rows ``c << chunk_shift``
    onwards; every chunk but the last has exactly 2^chunk_shift rows): this
    rank's own, a peer's mapped by IPC (GPU: each chunk is its own allocation
    and its own IPC object), or views of a peer's shared-memory file (CPU). A
    rank given as one tensor is one chunk. Table t is rows ``off[t] ..
    off[t] + rows[t]`` of ``stores[owner[t]]``."""

    def __init__(self, stores: Sequence, owner: Sequence[int], off: Sequence[int], rows: Sequence[int], rank: int,
                 chunk_shift: Optional[int] = None):
        self.stores = [[s] if isinstance(s, torch.Tensor) else list(s) for s in stores]
        self.owner, self.off, self.rows, self.rank = list(owner), list(off), list(rows), int(rank)
        self.T = len(self.owner)
        if chunk_shift is None:
            if all(len(c) == 1 for c in self.stores):
                chunk_shift = max(1, max(int(c[0].shape[0]) for c in self.stores) - 1).bit_length()
            else:
                chunk_shift = CHUNK_SHIFT
        self.chunk_shift = int(chunk_shift)
        per = 1 << self.chunk_shift
        total = []
        for r, chunks in enumerate(self.stores):
            for i, c in enumerate(chunks):
                if c.dim() != 2 or c.shape[1] != D or not c.is_contiguous():
                    raise ValueError("peer store chunks must be contiguous [rows, 64]")
                if c.shape[0] > per or (i < len(chunks) - 1 and c.shape[0] != per):
                    raise ValueError(f"rank {r} chunk {i}: {c.shape[0]} rows, chunks hold 2^{self.chunk_shift}")
            total.append(sum(int(c.shape[0]) for c in chunks))
        for t in range(self.T):
            if self.off[t] < 0 or self.off[t] + self.rows[t] > total[self.owner[t]]:
                raise ValueError(f"table {t}: rows {self.off[t]}..{self.off[t] + self.rows[t]} outside its owner's "
                                 f"store ({total[self.owner[t]]} rows)")
        mine = self.stores[self.rank][0]
        dev = mine.device
        self.dtype = mine.dtype
        maxc = max(len(c) for c in self.stores)
        i64 = dict(dtype=torch.int64, device=dev)
        self.trows = torch.tensor(self.rows, **i64)
        self.toff = torch.tensor(self.off, **i64)
        self.towner = torch.tensor(self.owner, dtype=torch.int32, device=dev)
        self.tremote = torch.tensor([int(o != self.rank) for o in self.owner], dtype=torch.int32, device=dev)
        self.cbase = torch.tensor([[c.data_ptr() for c in chunks] + [0] * (maxc - len(chunks))
                                   for chunks in self.stores], **i64)
        self._owner_cpu = torch.tensor(self.owner, dtype=torch.int64)
        self._off_cpu = torch.tensor(self.off, dtype=torch.int64)
        self.trows_cpu = torch.tensor(self.rows, dtype=torch.int64)
        self.tremote_cpu = self.tremote.cpu().bool()

    def kernel_args(self) -> dict:
        return dict(cbase=self.cbase, towner=self.towner, toff=self.toff, trows=self.trows, tremote=self.tremote,
                    chunk_shift=self.chunk_shift)

    @property
    def remote_tables(self) -> int:
        return int(self.tremote_cpu.sum())

    def row_cpu(self, t: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
        """Rows v of tables t (int64 [n] each) read from their owners' stores."""
        out = torch.empty(t.numel(), D, dtype=self.dtype)
        own = self._owner_cpu[t]
        g = self._off_cpu[t] + v
        chunk = g >> self.chunk_shift
        local = g & ((1 << self.chunk_shift) - 1)
        key = own * (1 << 20) + chunk
        for k in torch.unique(key).tolist():
            m = key == k
            out[m] = self.stores[k >> 20][k & ((1 << 20) - 1)][local[m]].cpu()
        return out


# Bytes of device memory one cached row costs: the bf16 row + its share of the
# two {key, slot} index buffers (2 x 2 entries x 16 B at the 50 % load factor)
# + the hot-set / candidate arrays of a refresh.
CACHE_BYTES_PER_ROW = 2 * D + 64 + 32


def auto_capacity(peer: "PeerTables", free_bytes: Optional[int] = None, fraction: float = 0.25,
                  floor: int = 1 << 16) -> int:
    """Default replica-cache capacity: ``fraction`` of the device memory still
    free once the tables are placed, capped at the remote rows there are to
    cache. MI355X: ~250 GB free beside a 2 x 38 GB sharded DLRM -> room for
    every remote row of the round-4 rehearsal tables; the cap keeps small
    models from reserving memory they cannot use."""
    remote_rows = int(sum(int(r) for r, rem in zip(peer.rows, peer.tremote_cpu.tolist()) if rem))
    if remote_rows == 0:
        return 0
    if free_bytes is None:
        dev = peer.trows.device
        free_bytes = torch.cuda.mem_get_info(dev)[0] if dev.type == "cuda" else 1 << 30
    fit = int(fraction * free_bytes) // CACHE_BYTES_PER_ROW
    return max(min(floor, remote_rows), min(remote_rows, fit))


_DEBUG = os.environ.get("DTFS_CACHE_DEBUG", "0") == "1"  # per-phase refresh timings (synchronizing)


def _member(x: torch.Tensor, sorted_set: torch.Tensor) -> torch.Tensor:
    """Bool mask: x[i] in sorted_set (one binary search per element; torch.isin
    re-sorts both inputs)."""
    if sorted_set.numel() == 0:
        return torch.zeros_like(x, dtype=torch.bool)
    pos = torch.searchsorted(sorted_set, x).clamp_(max=sorted_set.numel() - 1)
    return sorted_set[pos] == x


class HotRowCache:
    """This rank's replica of hot rows of tables owned by other ranks.

    ``capacity`` rows ([capacity, 64] bf16) behind two open-addressing index
    buffers ({key, slot} int64 entries [H, 2], H = the power of two >= 2 x
    capacity; one 16-byte load per probe): one serves the steps while
    :meth:`refresh` rebuilds the other.
    ``desc`` (int64 [5], read by the kernels at their start) = {active index,
    sample period, H - 1, rows, capacity}: a refresh changes only its first
    word (one 8-byte store), so a kernel sees the old index or the new one,
    whole; the sample period (0 = ``sample_every``) lets a learning phase
    sample every candidate without re-capturing the step's graphs.

    Slot safety: the rows a refresh adds go only into slots the CURRENT index
    does not reference, it keeps at most ``fill`` x capacity rows hot so there
    are free slots for the next turnover, and the index it rebuilds (the one
    the previous refresh replaced) must no longer be read by any step. With the
    serving step's stream registered (:meth:`set_step_stream`: the live
    server's StepRunner compute stream, where every kernel of a peer-exchange
    step runs) the refresh's kernels are enqueued on that stream, so stream
    order alone keeps them behind every step that could still read the old
    index and ahead of every step that reads the new one: no event, no
    device-wide synchronize, no stream of its own. (A side stream beside the
    steps stalled them for 10-30 s once refreshes ran while two ranks shared
    one GPU, profiles/r06_hot_cache_refresh.md.) The price is the refresh's own
    GPU time in the step stream, ~1.5 ms per refresh when the hot set did not
    change (the index is then left as it is) and a few ms when it did.
    Without a registered stream (tests, eager use) the refresh runs on a side
    stream after a device-wide synchronize."""

    def __init__(self, peer: PeerTables, capacity: Optional[int] = -1, ring_cap: Optional[int] = None,
                 sample_every: int = 8, decay: float = 0.5, fill: float = 0.75):
        self.peer = peer
        self.sized = "explicit"
        if capacity is None or int(capacity) < 0:  # auto: from the free device memory
            capacity, self.sized = auto_capacity(peer), "auto (a quarter of free device memory, capped at the remote rows)"
        self.cap = max(1, int(capacity))
        self.H = _next_pow2(2 * self.cap)
        self.sample_every, self.decay, self.fill = int(sample_every), float(decay), float(fill)
        dev = peer.trows.device
        self.device = dev
        if ring_cap is None:
            # the ring holds the keys sampled between two refreshes: 16 M on a
            # GPU (128 MB of its 288 GB) so a learning phase that samples every
            # candidate of tens of steps loses none; small on the CPU
            ring_cap = (1 << 24) if dev.type == "cuda" else (1 << 16)
        i64 = dict(dtype=torch.int64, device=dev)
        self.rows = torch.zeros(self.cap, D, dtype=peer.dtype, device=dev)
        self.index = [torch.full((self.H, 2), -1, **i64) for _ in range(2)]  # {key, slot} entries
        self.desc = torch.tensor([0, 0, self.H - 1, self.rows.data_ptr() if dev.type == "cuda" else 0, self.cap], **i64)
        self.stats = torch.zeros(128, **i64)
        self.ring = torch.full((max(64, -(-int(ring_cap) // 64) * 64),), -1, **i64)  # 64 segments
        self.ring_ctr = torch.zeros(64, **i64)
        self.keys = torch.empty(0, **i64)          # the active hot set, sorted
        self.slots = torch.empty(0, dtype=torch.int32, device=dev)
        self.cand_keys = torch.empty(0, **i64)     # candidates with decayed counts
        self.cand_score = torch.empty(0, dtype=torch.float32, device=dev)
        self.active = -1
        self.sample_period = 0
        self.refreshes = 0
        self.refresh_failures = 0
        self.last_error: Optional[str] = None
        self.last_filled = 0
        self._stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self._ordered = False  # set_step_stream: _stream IS the steps' stream
        self._lock = threading.Lock()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # -- kernel arguments -------------------------------------------------------
    def kernel_args(self) -> dict:
        return dict(cache=self.desc, stats=self.stats, ring=self.ring, ring_ctr=self.ring_ctr,
                    sample_every=self.sample_every)

    # -- counters ---------------------------------------------------------------
    def counts(self) -> Tuple[int, int]:
        """(hits, misses) of the counted remote lookups since the last reset:
        those of every ``sample_every``-th candidate, offset by half a period
        from the candidates whose keys are sampled for the hot set (all when
        ``sample_every`` <= 1); :attr:`count_scale` x these estimates the totals."""
        s = self.stats.view(64, 2).sum(0).cpu()
        return int(s[0]), int(s[1])

    @property
    def count_scale(self) -> int:
        return max(1, self.sample_every)

    def hit_rate(self) -> float:
        h, m = self.counts()
        return h / (h + m) if h + m else 0.0

    def reset_counts(self) -> None:
        self.stats.zero_()

    def set_sample_period(self, n: int = 0) -> None:
        """Sample the remote keys of every n-th candidate from the next step
        on (n = 1: all; 0: back to ``sample_every``). Kernels read it from the
        descriptor, so captured graphs need no re-capture."""
        self.desc[1:2].fill_(int(n))
        self.sample_period = int(n)

    # -- CPU reference of the kernels' cache side ---------------------------------
    def lookup_cpu(self, keys: torch.Tensor) -> torch.Tensor:
        """Slot of each key in the active set, -1 if absent."""
        k = self.keys.cpu()
        if k.numel() == 0:
            return torch.full_like(keys, -1, dtype=torch.int64)
        pos = torch.searchsorted(k, keys).clamp(max=k.numel() - 1)
        found = k[pos] == keys
        return torch.where(found, self.slots.cpu().long()[pos], torch.full_like(pos, -1))

    def count_cpu(self, hits: int, misses: int) -> None:
        self.stats[0] += hits
        self.stats[1] += misses

    def push_cpu(self, keys: torch.Tensor) -> None:
        """The kernels' ring push (one segment: the whole ring, counter 0)."""
        n = keys.numel()
        if n == 0:
            return
        cap = self.ring.numel()
        base = int(self.ring_ctr[0])
        pos = (torch.arange(n, dtype=torch.int64) + base) % cap
        self.ring[pos] = keys
        self.ring_ctr[0] = base + n

    # -- refresh ----------------------------------------------------------------
    @torch.no_grad()
    def refresh(self) -> int:
        """Fold the sampled keys into the counts and install the new hot set.
        Returns the number of rows copied in. Safe while steps run."""
        with self._lock:
            return self._refresh()

    def set_step_stream(self, stream_ptr: int) -> None:
        """Run refreshes on the raw HIP stream the serving steps run on (every
        kernel that reads the cache): stream-ordered with the steps."""
        if self.device.type == "cuda" and stream_ptr:
            self._stream = torch.cuda.ExternalStream(int(stream_ptr), device=self.device)
            self._ordered = True

    def _refresh(self) -> int:
        cuda = self.device.type == "cuda"
        dbg = _DEBUG and cuda
        marks = [("start", time.perf_counter())]

        def mark(what):
            if dbg:
                self._stream.synchronize()
                marks.append((what, time.perf_counter()))

        if cuda and not self._ordered:  # side stream: every step that may read the old index is done
            torch.cuda.synchronize(self.device)
            mark("sync")
        with (torch.cuda.stream(self._stream) if cuda else nullcontext()):
            samp = self.ring.clone()
            self.ring.fill_(-1)  # each refresh counts only the keys pushed since the last one
            self.ring_ctr.zero_()
            samp = samp[samp >= 0]
            if samp.numel():
                k, c = torch.unique(samp, return_counts=True)
                keys = torch.cat([self.cand_keys, k])
                score = torch.cat([self.cand_score * self.decay, c.float()])
                uk, inv = torch.unique(keys, return_inverse=True)
                s = torch.zeros(uk.numel(), dtype=torch.float32, device=self.device).scatter_add_(0, inv, score)
                top = torch.topk(s, min(uk.numel(), 4 * self.cap)).indices  # sorted by score
                self.cand_keys, self.cand_score = uk[top], s[top]
            mark("count")
            target = min(self.cand_keys.numel(), max(1, int(self.fill * self.cap)))
            hot = self.cand_keys[:target]
            hot_sorted = torch.sort(hot).values
            if self.active >= 0 and hot_sorted.numel() == self.keys.numel() and torch.equal(hot_sorted, self.keys):
                mark("same")
                self.refreshes += 1
                self.last_filled = 0
                if dbg:
                    print(f"[hot_cache] refresh {self.refreshes}: hot set unchanged "
                          f"({(time.perf_counter() - marks[0][1]) * 1e3:.2f} ms)", flush=True)
                return 0  # the active index already holds exactly this set
            kept = _member(self.keys, hot_sorted)  # self.keys is sorted
            kept_keys, kept_slots = self.keys[kept], self.slots[kept]
            new = hot[~_member(hot, self.keys)]  # hottest first
            mark("member")
            # free slots for the new rows among the first |new| + |active| slots:
            # at most |active| of those are referenced by the active index (not
            # writable now), so the window holds enough - O(hot set) work and
            # memory per refresh instead of O(capacity)
            window = min(self.cap, int(new.numel()) + int(self.slots.numel()))
            used = torch.zeros(window, dtype=torch.bool, device=self.device)
            if self.slots.numel() and window:
                act = self.slots.long()
                used[act[act < window]] = True
            free = (~used).nonzero().view(-1)
            mark("free")
            new = new[:free.numel()]
            new_slots = free[:new.numel()].to(torch.int32)
            if new.numel():
                self._fill(new, new_slots)
            keys = torch.cat([kept_keys, new])
            slots = torch.cat([kept_slots, new_slots])
            order = torch.argsort(keys)
            keys, slots = keys[order].contiguous(), slots[order].contiguous()
            mark("fill+sort")
            side = 0 if self.active != 0 else 1
            if cuda:
                idx = self.index[side]
                idx.fill_(-1)
                if keys.numel():
                    from ..ops import hip

                    hip().cache_index_build(keys, slots, idx)
                self.desc[0:1].fill_(self.index[side].data_ptr())  # one 8-byte store: the swap
            mark("index")
        if cuda:
            self._stream.synchronize()  # the swap's store has landed
        self.keys, self.slots = keys, slots
        self.active = side
        self.refreshes += 1
        self.last_filled = int(new.numel())
        if dbg:
            t = [(w, round((b - a) * 1e3, 2)) for (_, a), (w, b) in zip(marks, marks[1:])]
            print(f"[hot_cache] refresh {self.refreshes}: {t} ms, keys {int(keys.numel())}", flush=True)
        return self.last_filled

    def _fill(self, keys: torch.Tensor, slots: torch.Tensor) -> None:
        p = self.peer
        if self.device.type == "cuda":
            from ..ops import hip

            hip().peer_cache_fill(keys, slots, rows=self.rows, **p.kernel_args())
        else:
            t, v = keys >> KEY_SHIFT, keys & ROW_MASK
            self.rows[slots.long()] = p.row_cpu(t, v)

    # -- background refresh (serving) ---------------------------------------------
    def start(self, interval_s: float = 1.0) -> None:
        """Refresh every ``interval_s`` seconds on a daemon thread."""
        if self._thread is not None:
            return
        self._stop.clear()

        def loop():
            # a failed refresh leaves the previous hot set installed (the swap is
            # the refresh's last store) and is retried with exponential backoff;
            # failures and the thread's liveness are reported by describe() and
            # the live stats (serving/monitoring.py)
            wait = interval_s
            while not self._stop.wait(wait):
                try:
                    self.refresh()
                    wait = interval_s
                except Exception as e:  # the cache is an optimisation: keep serving
                    self.refresh_failures += 1
                    self.last_error = repr(e)
                    wait = min(60.0, max(interval_s, wait * 2))
                    print(f"[hot_cache] refresh failed ({self.refresh_failures}), retrying in {wait:.1f} s: {e!r}",
                          flush=True)

        self._thread = threading.Thread(target=loop, name="dtfs-hot-cache", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=30)
            self._thread = None

    @property
    def refresher_alive(self) -> bool:
        return self._thread is not None and self._thread.is_alive()

    def describe(self) -> dict:
        h, m = self.counts()
        return {"capacity_rows": self.cap, "sized": self.sized, "hot_rows": int(self.keys.numel()),
                "refreshes": self.refreshes,
                "hits": h, "misses": m, "hit_rate": round(h / (h + m), 4) if h + m else None,
                "refresh_failures": self.refresh_failures, "refresher_alive": self.refresher_alive,
                "last_error": self.last_error}


def peer_gather_cpu(peer: PeerTables, cache: Optional[HotRowCache], ids: torch.Tensor, wts: Optional[torch.Tensor],
                    hot: int) -> torch.Tensor:
    """CPU reference of the peer lookup (kernels/peer_lookup.h): ids [B, T *
    hot] (table t's bag = columns t * hot .. + hot - 1), wts the same shape for
    bags (None: one-hot) -> bf16 [B, T, 64]; counts and samples like the kernels."""
    B, T = ids.shape[0], peer.T
    t = torch.arange(T, dtype=torch.int64).repeat_interleave(hot).view(1, -1).expand(B, -1).reshape(-1)
    v = torch.remainder(ids.long().reshape(-1), peer.trows_cpu[t])
    rows = peer.row_cpu(t, v).float()
    if cache is not None:
        remote = peer.tremote_cpu[t]
        keys = (t << KEY_SHIFT) | v
        slot = cache.lookup_cpu(keys)
        hit = remote & (slot >= 0)
        if bool(hit.any()):
            rows[hit] = cache.rows.cpu()[slot[hit]].float()
        b = torch.arange(B, dtype=torch.int64).repeat_interleave(T * hot)
        n = cache.sample_every
        sp = cache.sample_period if cache.sample_period > 0 else n  # the kernels' peer_sample_period
        sampled = (b % sp == 0) if sp > 1 else torch.ones_like(b, dtype=torch.bool)
        counted = (b % n == n // 2) if n > 1 else torch.ones_like(b, dtype=torch.bool)
        cache.count_cpu(int((hit & counted).sum()), int((remote & ~hit & counted).sum()))
        if n > 0:
            cache.push_cpu(keys[remote & sampled])
    if wts is None:
        out = rows.view(B, T, D)
    else:
        out = (rows.view(B, T, hot, D) * wts.float().reshape(B, T, hot, 1)).sum(2)
    return out.to(peer.dtype)


def open_peer_stores(chunks: List[torch.Tensor], group=None, shm_tag: Optional[str] = None,
                     chunk_shift: Optional[int] = None) -> List[List[torch.Tensor]]:
    """Every rank's store chunks as seen from this rank (collective). GPU:
    one IPC handle per chunk (each chunk its own allocation, see
    :func:`alloc_store`) exchanged with all_gather_object, each peer chunk
    mapped for loads over xGMI. CPU: the chunks are views of one
    shared-memory file made by :func:`alloc_store`, ``shm_tag`` its path."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    chunk_shift = CHUNK_SHIFT if chunk_shift is None else chunk_shift
    if world == 1:
        return [chunks]
    cuda = chunks[0].is_cuda
    if cuda:
        from ..ops import hip

        mine = [(*hip().ipc_export(c), list(c.shape)) for c in chunks]
    else:
        if shm_tag is None:
            raise ValueError("CPU peer stores need their shared-memory tag")
        mine = [(shm_tag, 0, [sum(int(c.shape[0]) for c in chunks), D])]
    allv: list = [None] * world
    dist.all_gather_object(allv, mine, group=group)
    out: List[List[torch.Tensor]] = []
    for r, theirs in enumerate(allv):
        if r == rank:
            out.append(list(chunks))
        elif cuda:
            from ..ops import hip

            out.append([hip().ipc_open(h, off, shape, chunks[0]) for h, off, shape in theirs])
        else:
            path, _, shape = theirs[0]
            whole = torch.from_file(path, shared=True, size=int(shape[0]) * D, dtype=chunks[0].dtype).view(*shape)
            out.append(list(torch.split(whole, 1 << chunk_shift)))
    dist.barrier(group=group)  # every rank has mapped every chunk: the file names can go
    return out


def alloc_store(rows: int, dtype, device, shm_tag: Optional[str] = None,
                chunk_shift: Optional[int] = None) -> List[torch.Tensor]:
    """A store of ``rows`` [64]-wide rows as chunks of 2^chunk_shift rows.
    GPU: each chunk is its own hipMalloc allocation (a peer maps exactly that
    chunk); CPU: views of one shared-memory file other ranks can map."""
    rows = max(1, int(rows))
    per = 1 << (CHUNK_SHIFT if chunk_shift is None else chunk_shift)
    if torch.device(device).type == "cuda":
        from ..ops import hip

        like = torch.empty(0, device=device)
        out = []
        for c0 in range(0, rows, per):
            n = min(per, rows - c0)
            out.append(hip().device_alloc(n * D * torch.tensor([], dtype=dtype).element_size(), like)
                       .view(dtype).view(n, D))
        return out
    if shm_tag is None:
        return list(torch.split(torch.empty(rows, D, dtype=dtype), per))
    whole = torch.from_file(shm_tag, shared=True, size=rows * D, dtype=dtype).view(rows, D)
    return list(torch.split(whole, per))

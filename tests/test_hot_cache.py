"""Peer exchange + hot-row replica cache (parallel/hot_cache.py): the sharded
DLRM reading each table where it lives (shared-memory stores on the CPU, IPC
over xGMI on the GPU) scores exactly like the unsharded model at world 2 / 3,
one-hot and multi-hot, before and after the cache fills from online counts;
the cache's refresh never writes a slot the live index references."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.parallel.hot_cache import KEY_SHIFT, HotRowCache, PeerTables, peer_gather_cpu


def _cfg(hot: int = 1, rows: int = 997):
    if hot > 1:
        return ModelConfig(family="dlrm", num_fields=5 + 5 * hot, num_dense=5, table_rows=rows, embed_dim=64,
                           bottom_mlp=(32, 64), mlp_dims=(64, 32), multi_hot=hot, embedding_exchange="peer",
                           hot_cache_rows=1024)
    return ModelConfig(family="dlrm", num_fields=20, num_dense=5, table_rows=rows, embed_dim=64,
                       bottom_mlp=(32, 64), mlp_dims=(64, 32), embedding_exchange="peer", hot_cache_rows=1024)


def _skewed(B, F, gen, hot_ids=40):
    """ids mostly drawn from a few hot values (the cache has something to hold)."""
    ids = torch.randint(0, 10**12, (B, F), generator=gen)
    hot = torch.randint(0, hot_ids, (B, F), generator=gen)
    pick = torch.rand(B, F, generator=gen) < 0.8
    return torch.where(pick, hot, ids)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, hot, q, chunk_shift=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.parallel.dist import init_from_env, shutdown
    from distributed_tf_serving_amd.parallel.embedding_sharding import ShardedDLRM

    try:
        if chunk_shift is not None:  # stores split into many small chunks
            from distributed_tf_serving_amd.parallel import hot_cache

            hot_cache.CHUNK_SHIFT = chunk_shift
        ctx = init_from_env(device="cpu")
        cfg = _cfg(hot)
        m = ShardedDLRM(cfg, ctx)
        if chunk_shift is not None:
            assert m.emb.peer.chunk_shift == chunk_shift and len(m.emb.peer.stores[1 - rank]) > 10
        ref = build_model(cfg)
        assert not m.has_collectives and m.emb.exchange == "peer" and m.cache is not None
        m.cache.sample_every = 1  # small batches: sample every candidate
        g = torch.Generator().manual_seed(11 + rank)
        errs, rates = [], []
        for it in range(3):
            B = 24
            ids = _skewed(B, cfg.num_fields, g)
            wts = torch.rand(B, cfg.num_fields, generator=g)
            m.cache.reset_counts()
            out = m(ids, wts)
            errs.append((out - ref(ids, wts)).abs().max().item())
            rates.append(m.cache.hit_rate())
            m.cache.refresh()
        q.put((rank, max(errs), rates, m.cache.describe(), m.exchange_bytes(24)))
        shutdown()
    except Exception:  # pragma: no cover - surfaced by the assertion below
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None))


@pytest.mark.slow
@pytest.mark.parametrize("world,hot,chunk_shift", [(2, 1, None), (3, 1, None), (2, 3, None), (2, 1, 6)])
def test_peer_exchange_matches_unsharded(world, hot, chunk_shift):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, hot, q, chunk_shift)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world):
        r, err, rates, desc, xb = q.get(timeout=240)
        res[r] = (err, rates, desc, xb)
    [p.join(timeout=60) for p in procs]
    for r in range(world):
        err, rates, desc, xb = res[r]
        assert isinstance(err, float), f"rank {r} failed: {err}"
        assert err < 1e-5, f"rank {r}: peer-exchange scores differ by {err}"
        assert rates[0] == 0.0  # nothing cached before the first refresh
        assert rates[-1] > 0.3, rates  # the hot ids are served from the replica
        assert desc["hot_rows"] > 0 and desc["refreshes"] == 3
        assert xb > 0


def _local_peer(T=4, rows=50, remote=(1, 3), chunk_shift=None):
    """Two 'ranks' in one process: tables in `remote` live in store 1
    (chunk_shift: each store split into chunks of 2^chunk_shift rows)."""
    torch.manual_seed(0)
    stores = [torch.randn(T * rows, 64).to(torch.bfloat16), torch.randn(T * rows, 64).to(torch.bfloat16)]
    if chunk_shift is not None:
        stores = [list(torch.split(s, 1 << chunk_shift)) for s in stores]
    owner = [1 if t in remote else 0 for t in range(T)]
    off = [t * rows for t in range(T)]
    return PeerTables(stores, owner, off, [rows] * T, rank=0, chunk_shift=chunk_shift)


def test_chunked_store_rows():
    """Rows read through 16-row chunks equal the rows of the whole store."""
    whole, chunked = _local_peer(), _local_peer(chunk_shift=4)
    assert chunked.chunk_shift == 4 and len(chunked.stores[1]) == 13
    t = torch.arange(4).repeat_interleave(50)
    v = torch.arange(50).repeat(4)
    assert torch.equal(whole.row_cpu(t, v), chunked.row_cpu(t, v))
    with pytest.raises(ValueError):  # a middle chunk must hold exactly 2^shift rows
        PeerTables([[torch.zeros(8, 64), torch.zeros(16, 64)]], [0], [0], [20], rank=0, chunk_shift=4)


def test_auto_capacity_from_free_memory():
    """Default capacity: a quarter of the free device memory at
    CACHE_BYTES_PER_ROW a row, capped at the remote rows (floor 64 k or all of
    them); no remote table, no cache."""
    from distributed_tf_serving_amd.parallel.hot_cache import CACHE_BYTES_PER_ROW, auto_capacity

    p = _local_peer(T=4, rows=50, remote=(1, 3))
    assert auto_capacity(p, free_bytes=1 << 40) == 100  # capped: 2 remote tables x 50 rows
    assert auto_capacity(_local_peer(remote=())) == 0
    big = _local_peer(T=2, rows=50, remote=(1,))
    big.rows = [50, 10 ** 9]  # a billion-row remote table (the stores stay small: capacity math only)
    assert auto_capacity(big, free_bytes=4 * CACHE_BYTES_PER_ROW * 10 ** 6) == 10 ** 6
    assert auto_capacity(big, free_bytes=0) == 1 << 16  # the floor
    c = HotRowCache(p, capacity=-1, ring_cap=64)
    assert c.cap == 100 and c.describe()["sized"].startswith("auto")
    assert HotRowCache(p, capacity=8, ring_cap=64).describe()["sized"] == "explicit"


def test_cache_refresh_slot_safety_and_turnover():
    p = _local_peer()
    c = HotRowCache(p, capacity=8, ring_cap=64, sample_every=1, fill=0.75)
    # round 1: keys of tables 1 and 3 rows 0..9, rows 0..5 much hotter
    ids = torch.tensor([[r % 6 if i % 3 else r % 10 for i in range(4)] for r in range(30)])
    peer_gather_cpu(p, c, ids, None, 1)
    assert c.counts() == (0, 60)  # 2 remote tables x 30 rows, all misses
    assert c.refresh() == 6 and c.keys.numel() == 6  # fill 0.75 x 8
    hot1 = set(c.keys.tolist())
    slots1 = set(c.slots.tolist())
    # cached rows equal their owner's rows
    t, v = c.keys >> KEY_SHIFT, c.keys & ((1 << KEY_SHIFT) - 1)
    assert torch.equal(c.rows[c.slots.long()], p.row_cpu(t, v))
    c.reset_counts()
    out = peer_gather_cpu(p, c, ids, None, 1)
    h, m = c.counts()
    assert h > 0 and h + m == 60
    # the lookup reads the same bytes with or without the cache
    assert torch.equal(out, peer_gather_cpu(p, None, ids, None, 1))
    # round 2: a new hot set - new rows only go to slots the live index did not use
    ids2 = torch.full((40, 4), 33)
    ids2[:, 1] = torch.arange(40) % 4 + 20
    for _ in range(3):
        peer_gather_cpu(p, c, ids2, None, 1)
    n_new = c.refresh()
    assert 0 < n_new <= 8 - len(slots1)
    new_keys = set(c.keys.tolist()) - hot1
    new_slots = {s for k, s in zip(c.keys.tolist(), c.slots.tolist()) if k in new_keys}
    assert new_slots and not (new_slots & slots1)
    assert torch.equal(peer_gather_cpu(p, c, ids2, None, 1), peer_gather_cpu(p, None, ids2, None, 1))


def test_refresher_retries_failures_and_reports_them(monkeypatch):
    """A failing refresh keeps the last hot set, is counted, and is retried
    with backoff by a refresher that stays alive (it used to exit for good on
    the first exception, leaving a silently frozen cache)."""
    import time

    p = _local_peer()
    c = HotRowCache(p, capacity=8, ring_cap=64, sample_every=1)
    calls = {"n": 0}
    real = c._refresh

    def flaky():
        calls["n"] += 1
        if calls["n"] <= 2:
            raise RuntimeError("injected refresh failure")
        return real()

    monkeypatch.setattr(c, "_refresh", flaky)
    c.start(interval_s=0.01)
    try:
        t0 = time.time()
        while c.refreshes == 0 and time.time() - t0 < 10:
            time.sleep(0.01)
        d = c.describe()
        assert d["refresh_failures"] == 2 and d["refresher_alive"] and c.refreshes >= 1
        assert "injected" in d["last_error"]
    finally:
        c.stop()
    assert not c.describe()["refresher_alive"]


def test_local_tables_never_cached_or_counted():
    p = _local_peer(remote=())
    assert p.remote_tables == 0
    c = HotRowCache(p, capacity=4, sample_every=1)
    peer_gather_cpu(p, c, torch.zeros(8, 4, dtype=torch.int64), None, 1)
    assert c.counts() == (0, 0) and int(c.ring_ctr.sum()) == 0


# ---------------------------------------------------------------------- GPU
def _gpu_peer(dev, T=6, rows=4096, remote=(1, 2, 4), chunk_shift=None):
    g = torch.Generator(device="cpu").manual_seed(3)
    stores = [torch.randn(T * rows, 64, generator=g).to(torch.bfloat16).to(dev) for _ in range(2)]
    if chunk_shift is not None:  # chunks = views of the store; the kernels only see chunk addresses
        stores = [list(torch.split(s, 1 << chunk_shift)) for s in stores]
    owner = [1 if t in remote else 0 for t in range(T)]
    return PeerTables(stores, owner, [t * rows for t in range(T)], [rows] * T, rank=0, chunk_shift=chunk_shift)


def _cpu_twin(p):
    return PeerTables([[c.cpu() for c in s] for s in p.stores], p.owner, p.off, p.rows, p.rank, p.chunk_shift)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_shift", [None, 9])
def test_peer_kernels_match_reference(cuda, chunk_shift):
    from distributed_tf_serving_amd import ops

    p = _gpu_peer(cuda, chunk_shift=chunk_shift)
    pc = _cpu_twin(p)
    T, B, col0 = p.T, 1000, 3
    g = torch.Generator().manual_seed(5)
    ids = _skewed(B, col0 + T * 2, g, hot_ids=64)
    wts = torch.rand(B, col0 + T * 2, generator=g)
    dense = torch.randn(B, 64, generator=g).to(torch.bfloat16)
    c = HotRowCache(p, capacity=2048, ring_cap=1 << 14, sample_every=2)
    cc = HotRowCache(pc, capacity=2048, ring_cap=1 << 14, sample_every=2)
    for rnd in range(2):
        c.reset_counts()
        cc.reset_counts()
        z = ops.dot_interaction_gather_peer(dense.to(cuda), ids.to(cuda), p, c, id_col0=col0)
        zr = ops.dot_interaction_gather_peer(dense, ids, pc, cc, id_col0=col0)
        torch.cuda.synchronize()
        assert (z.float().cpu() - zr.float()).abs().max().item() < 2e-2 * max(1.0, zr.float().abs().max().item())
        bag = ops.peer_bag(ids.to(cuda), wts.to(cuda), B, col0, 2, p, c)
        bagr = ops.peer_bag(ids, wts, B, col0, 2, pc, cc)
        torch.cuda.synchronize()
        assert (bag.float().cpu() - bagr.float()).abs().max().item() < 1e-2
        h, m = c.counts()
        hr, mr = cc.counts()
        # every 2nd candidate counted: 3 remote tables, (1 one-hot + 2 bag) lookups each
        assert h + m == hr + mr == (B // 2) * 3 * 3
        if rnd == 0:
            assert h == 0
            assert int(c.ring_ctr.sum()) == int(cc.ring_ctr.sum()) == (B // 2) * 3 * 3
            assert c.refresh() > 0 and cc.refresh() > 0
            # the GPU index finds every hot key at its slot
            assert torch.equal(c.keys.cpu(), cc.keys.cpu())
        else:
            assert h == hr > 0


@pytest.mark.gpu
def test_ipc_export_open_same_process(cuda):
    from distributed_tf_serving_amd.ops import hip

    x = torch.arange(4096, dtype=torch.float32, device=cuda).view(64, 64)
    y = x[8:]
    h, off = hip().ipc_export(y)
    assert off >= 8 * 64 * 4 and isinstance(h, bytes)


@pytest.mark.gpu
@pytest.mark.parametrize("ordered", [False, True])
def test_refresh_while_lookups_run(cuda, ordered):
    """Refreshes (new rows copied into free slots, the other index built and
    swapped in by one 8-byte store) while another thread keeps launching
    cached lookups on its own stream, four in flight at a time: every lookup
    returns exactly the rows of the uncached lookup, through hot-set turnover.
    ordered: the lookups' stream is registered (set_step_stream, as the live
    server registers its compute stream) and the refreshes run on it,
    stream-ordered with the lookups, instead of on a side stream after a
    device-wide synchronize."""
    import threading
    import time

    from distributed_tf_serving_amd import ops

    p = _gpu_peer(cuda, chunk_shift=9)
    c = HotRowCache(p, capacity=1024, ring_cap=1 << 14, sample_every=2)
    g = torch.Generator().manual_seed(9)
    B, T = 2048, p.T
    # three batches whose hot ids differ: the hot set turns over as the mix shifts
    batches = [(_skewed(B, T, g, hot_ids=48) + 100 * k).to(cuda) for k in range(3)]
    dense = torch.randn(B, 64, generator=g).to(torch.bfloat16).to(cuda)
    want = [ops.dot_interaction_gather_peer(dense, ids, p, None) for ids in batches]
    torch.cuda.synchronize()
    s = torch.cuda.Stream(cuda)
    if ordered:
        c.set_step_stream(s.cuda_stream)
    stop, errs, done = threading.Event(), [], [0]

    def worker():
        k = 0
        with torch.cuda.stream(s):
            while not stop.is_set():
                zs = [(k + j, ops.dot_interaction_gather_peer(dense, batches[(k + j) % 3], p, c)) for j in range(4)]
                s.synchronize()
                errs.extend(i for i, z in zs if not torch.equal(z, want[i % 3]))
                k += 4
        done[0] = k

    t = threading.Thread(target=worker)
    t.start()
    try:
        for _ in range(12):
            time.sleep(0.02)
            c.refresh()
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errs, errs[:5]
    assert done[0] > 12 and c.refreshes == 12 and c.keys.numel() > 0
    assert c._ordered == ordered
    h, m = c.counts()
    assert h > 0

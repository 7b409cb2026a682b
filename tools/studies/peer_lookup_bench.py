"""Kernel-level cost of the peer lookup on one GPU (one process): the DLRM
interaction of 16384 candidates x 26 one-hot tables, rows gathered

* ``local``: from one store (``dot_interaction_gather``, the one-rank step);
* ``peer``: through the peer lookup (chunked stores, per-table owner, half the
  tables "remote" in a second store of the same GPU), no replica cache;
* ``peer+cache``: the same after the replica cache learned the stream.

On one GPU the "remote" store is local HBM, so this measures the lookup's own
overhead (chunk addressing, cache probes, counters, sampling), not xGMI.
Prints one JSON line."""
from __future__ import annotations

import argparse
import json

import numpy as np
import torch


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000, help="rows per table")
    ap.add_argument("--tables", type=int, default=26)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--cache-rows", type=int, default=1 << 20)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from distributed_tf_serving_amd import ops
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.parallel.hot_cache import CHUNK_SHIFT, HotRowCache, PeerTables, alloc_store

    dev = torch.device("cuda", 0)
    T, R, B = a.tables, a.rows, a.batch
    half = T // 2
    # rank 0 owns tables [0, half), "rank 1" the rest; both stores on this GPU
    own = [0 if t < half else 1 for t in range(T)]
    n0, n1 = half * R, (T - half) * R
    stores = [alloc_store(n0, torch.bfloat16, dev), alloc_store(n1, torch.bfloat16, dev)]
    for chunks in stores:
        for c in chunks:
            c.uniform_(-0.05, 0.05)
    off = [t * R if t < half else (t - half) * R for t in range(T)]
    peer = PeerTables(stores, own, off, [R] * T, rank=0, chunk_shift=CHUNK_SHIFT)
    # the local form: every table in one [T x R, 64] store (separate buffer, same values not needed)
    local = torch.empty(T * R, 64, dtype=torch.bfloat16, device=dev).uniform_(-0.05, 0.05)
    modf = torch.full((T,), R, dtype=torch.int64, device=dev)
    offf = torch.arange(T, dtype=torch.int64, device=dev) * R
    synth = SyntheticRequests(fields=T, id_space=1 << 40, dist="zipf", seed=5)
    batches = [torch.from_numpy(synth.arrays(B)[0]).to(dev) for _ in range(8)]
    dense = torch.randn(B, 64, device=dev).to(torch.bfloat16)

    def timed(fn) -> float:
        for i in range(5):
            fn(batches[i % len(batches)])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(a.iters):
            fn(batches[i % len(batches)])
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    out = {"batch": B, "tables": T, "rows_per_table": R, "remote_tables": T - half}
    out["local_us"] = round(timed(lambda ids: ops.dot_interaction_gather(dense, local, ids, modf, offf)), 2)
    out["peer_us"] = round(timed(lambda ids: ops.dot_interaction_gather_peer(dense, ids, peer)), 2)
    cache = HotRowCache(peer, a.cache_rows, sample_every=8)
    for _ in range(4):  # learn the stream
        for ids in batches:
            ops.dot_interaction_gather_peer(dense, ids, peer, cache)
        cache.refresh()
    cache.reset_counts()
    out["peer_cache_us"] = round(timed(lambda ids: ops.dot_interaction_gather_peer(dense, ids, peer, cache)), 2)
    h, m = cache.counts()
    from distributed_tf_serving_amd.ops import hip

    # the same lookups without the counters / sampling, and the counters alone
    out["peer_cache_no_counters_us"] = round(timed(lambda ids: hip().dot_interaction_gather_peer(
        dense, ids, None, 0, cache=cache.desc, **peer.kernel_args())), 2)
    out["peer_counters_only_us"] = round(timed(lambda ids: hip().dot_interaction_gather_peer(
        dense, ids, None, 0, stats=cache.stats, ring=cache.ring, ring_ctr=cache.ring_ctr, sample_every=8,
        **peer.kernel_args())), 2)
    out["peer_stats_only_us"] = round(timed(lambda ids: hip().dot_interaction_gather_peer(
        dense, ids, None, 0, stats=cache.stats, **peer.kernel_args())), 2)
    out["hit_rate"] = round(h / max(1, h + m), 4)
    out["hot_rows"] = int(cache.keys.numel())
    # the same hot set on a fresh draw of the stream
    fresh = synth.arrays(B)[0].astype(np.int64) % R
    keys = cache.keys.cpu().numpy()
    hit = tot = 0
    for t in range(half, T):
        k = (np.int64(t) << 40) | fresh[:, t]
        pos = np.clip(np.searchsorted(keys, k), 0, max(0, keys.size - 1))
        hit += int((keys[pos] == k).sum()) if keys.size else 0
        tot += k.size
    out["hit_rate_fresh_stream"] = round(hit / max(1, tot), 4)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    cache.refresh()
    t1.record()
    torch.cuda.synchronize()
    out["refresh_ms"] = round(t0.elapsed_time(t1), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

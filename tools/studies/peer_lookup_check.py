"""Peer exchange check on N ranks (torchrun; on a 1-GPU box with
DTFS_SHARE_GPU=1 the ranks share the card and map each other's stores by IPC
exactly as 8 GPUs do over xGMI): the sharded DLRM reading every table where it
lives scores like the unsharded DLRM of the same seed - one-hot (the fused
interaction kernel) and multi-hot bags - before and after the hot-row replica
cache fills, through the eager forward and through the arena step program.
Rank 0 prints one JSON line."""
from __future__ import annotations

import argparse
import json
import sys

import torch
import torch.distributed as dist


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20011)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--hot", type=int, default=1)
    a = ap.parse_args()
    from distributed_tf_serving_amd import ops
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.parallel.dist import init_from_env
    from distributed_tf_serving_amd.parallel.embedding_sharding import ShardedDLRM
    from distributed_tf_serving_amd.serving.arena import ArenaLayout

    ctx = init_from_env()
    dev = ctx.device

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    T = 8
    cfg = ModelConfig(family="dlrm", num_fields=13 + T * a.hot, num_dense=13, table_rows=a.rows, embed_dim=64,
                      multi_hot=a.hot, embedding_exchange="peer", hot_cache_rows=4096)
    m = ShardedDLRM(cfg, ctx, device=dev)
    ref = build_model(cfg, dev)  # the unsharded DLRM, same seed
    cache = m.cache
    assert cache is not None and not m.has_collectives
    cache.sample_every = 1
    synth = SyntheticRequests(fields=cfg.num_fields, id_space=1 << 40, dist="zipf", seed=17 + ctx.rank)
    res = {"world": ctx.world, "hot": a.hot, "remote_tables": m.emb.peer.remote_tables, "rounds": []}
    F = cfg.num_fields
    for rnd in range(3):
        ids_np, wts_np = synth.arrays(a.batch)
        ids, wts = torch.from_numpy(ids_np).to(dev), torch.from_numpy(wts_np).to(dev)
        cache.reset_counts()
        got = m(ids, wts)
        want = ref(ids, wts)
        sync()
        err = (got.float() - want.float()).abs().max().item()
        # the arena step program (K0 fused: ids read from the request bytes)
        A = ArenaLayout(F, a.batch)
        ar = A.alloc()
        reqs = [synth.serialized(a.batch // 4) for _ in range(4)]
        ab = A.build(ar, A.place(ar, reqs))
        assert not any(ab.errors)
        from distributed_tf_serving_amd.parallel import step_program as sp

        B = a.batch
        bufs = m.alloc(B)
        out = torch.zeros(B, device=dev)
        dev_ar = ar.to(dev)
        prog = m.build_program(ops.ArenaRows(dev_ar, B, F), None, B, bufs, out=out)
        sp.run_eager(prog, None)
        from distributed_tf_serving_amd.serving.packing import PackedLayout

        L = PackedLayout(F)
        packed = A.unpack_cpu(ar, L.alloc(B))
        want_a = ref(L.ids(packed).to(dev), L.wts(packed).to(dev))
        sync()
        err_a = (out.float() - want_a.float()).abs().max().item()
        h, mi = cache.counts()
        res["rounds"].append({"max_abs_diff": err, "max_abs_diff_arena_program": err_a, "hits": h, "misses": mi})
        cache.refresh()
    res["cache"] = cache.describe()
    allres = [None] * ctx.world
    dist.all_gather_object(allres, res)
    if ctx.rank == 0:
        print(json.dumps({"ranks": allres}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

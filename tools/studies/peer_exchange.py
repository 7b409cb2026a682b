"""One-shot peer exchange (csrc/kernels/peer.hip) vs RCCL: correctness and latency.

Run one process per rank (``torch.distributed.run``); on a 1-GPU box with
``DTFS_SHARE_GPU=1`` every rank shares the card (RCCL then uses its socket
transport while the peer kernel writes through IPC-mapped device memory, so
the latency columns are a rehearsal, not xGMI numbers). Each rank:

1. creates an RCCL communicator and a second one with the peer exchange on;
2. checks alltoall / allgather / gather / scatter of random bytes - including
   message sizes that are not multiples of 4 or 16 - on both against the
   expected layout (every rank knows every rank's seeded payload);
3. times ``--iters`` back-to-back exchanges per size on each (stream-ordered,
   one sync), max over ranks;
4. with ``--fault`` the last rank skips one exchange: the others must report
   the timeout through ``async_error()`` instead of hanging.

Rank 0 prints one JSON line. Reference counterpart: the per-shard RPC fan-out
and join the latency of which DCNClient.java:198-202 prints.
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.distributed as dist

from distributed_tf_serving_amd.parallel.dist import init_from_env
from distributed_tf_serving_amd.parallel.native_comm import create_comm


def payload(rank: int, peer: int, n: int, seed: int, dev) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed * 1_000_003 + rank * 1009 + peer)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(dev)


def check(comm, world: int, rank: int, n: int, seed: int, dev) -> None:
    # alltoall: recv[p] = p's message for me
    send = torch.cat([payload(rank, p, n, seed, dev) for p in range(world)])
    recv = torch.empty_like(send)
    comm.alltoall(send, recv)
    want = torch.cat([payload(p, rank, n, seed, dev) for p in range(world)])
    torch.cuda.synchronize()
    assert torch.equal(recv, want), f"alltoall n={n}"
    # allgather: recv[p] = p's message (peer index -1)
    mine = payload(rank, -1, n, seed + 1, dev)
    got = torch.empty(world * n, dtype=torch.uint8, device=dev)
    comm.allgather(mine, got)
    want = torch.cat([payload(p, -1, n, seed + 1, dev) for p in range(world)])
    torch.cuda.synchronize()
    assert torch.equal(got, want), f"allgather n={n}"
    for root in {0, world - 1}:
        g = torch.zeros(world * n if rank == root else 1, dtype=torch.uint8, device=dev)
        comm.gather(mine, g, root)
        torch.cuda.synchronize()
        if rank == root:
            assert torch.equal(g, want), f"gather n={n} root={root}"
        sc = torch.cat([payload(root, p, n, seed + 2, dev) for p in range(world)]) if rank == root else \
            torch.zeros(1, dtype=torch.uint8, device=dev)
        r = torch.zeros(n, dtype=torch.uint8, device=dev)
        comm.scatter(sc, r, root)
        torch.cuda.synchronize()
        assert torch.equal(r, payload(root, rank, n, seed + 2, dev)), f"scatter n={n} root={root}"


def time_op(comm, world: int, n: int, iters: int, dev) -> float:
    send = torch.zeros(world * n, dtype=torch.uint8, device=dev)
    recv = torch.empty_like(send)
    for _ in range(5):
        comm.alltoall(send, recv)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.alltoall(send, recv)
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) * 1e6 / iters], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return round(float(t.item()), 2)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--sizes", default="1,13,2048,6000,65536", help="bytes per peer (checked and timed)")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--timeout-s", type=float, default=5.0)
    ap.add_argument("--fault", action="store_true", help="last rank skips an exchange; the others must time out")
    ap.add_argument("--deny-access", action="store_true",
                    help="the last rank reports no peer access to the others: every rank must fall back to RCCL")
    a = ap.parse_args(argv)
    ctx = init_from_env()
    dev, rank, world = ctx.device, ctx.rank, ctx.world
    if world < 2 or not dist.is_initialized():
        raise SystemExit("run with torch.distributed.run and >= 2 ranks")
    sizes = [int(s) for s in a.sizes.split(",")]
    cap = max(sizes)
    # (ranks sharing one GPU in the rehearsal all report the same device: the
    # hook denies every pair, its own device included)
    deny = (lambda d: False) if (a.deny_access and rank == world - 1) else None
    peer = create_comm(ctx, peer_cap=cap, peer_timeout_s=a.timeout_s, can_access=deny)
    out = {"world": world}
    if a.deny_access:
        assert not peer.peer_enabled, "one rank had no peer access: the peer path must stay off everywhere"
        for i, n in enumerate(sizes):
            check(peer, world, rank, n, 300 + i, dev)
        assert peer.peer_exchanges == 0 and peer.async_error() == ""
        out.update(fallback="rccl", checked_sizes=sizes)
        dist.barrier()
        if rank == 0:
            print(json.dumps(out), flush=True)
        return 0
    assert peer.peer_enabled and peer.peer_cap >= cap
    out["cap"] = peer.peer_cap
    if a.fault:
        x = torch.zeros(world * 64, dtype=torch.uint8, device=dev)
        y = torch.empty_like(x)
        peer.alltoall(x, y)  # one good exchange
        torch.cuda.synchronize()
        if rank != world - 1:
            peer.alltoall(x, y)  # the last rank never joins this one
            t0 = time.perf_counter()
            torch.cuda.synchronize()  # bounded: the kernel gives up after timeout_s
            waited = time.perf_counter() - t0
            err = peer.async_error()
            assert "timed out" in err, err
            out.update(fault_detected=True, waited_s=round(waited, 2), error=err)
        dist.barrier()
        if rank == 0:
            print(json.dumps(out), flush=True)
        return 0
    rccl = create_comm(ctx, peer_cap=0)
    for i, n in enumerate(sizes):
        check(peer, world, rank, n, 100 + i, dev)
        check(rccl, world, rank, n, 200 + i, dev)
    assert peer.async_error() == "" and peer.peer_exchanges > 0
    out["checked_sizes"] = sizes
    out["alltoall_us"] = {str(n): {"peer": time_op(peer, world, n, a.iters, dev),
                                   "rccl": time_op(rccl, world, n, a.iters, dev)} for n in sizes}
    dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""Bootstrap of the native RCCL communicators (csrc/comm/rccl_comm.cpp).

torch.distributed is used once, to broadcast rank 0's 128-byte ncclUniqueId;
after that the fan-out collectives are issued from C++ by the StepRunner
(reference counterpart: the per-host channel setup, DCNClient.java:118-125).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import hip
from .dist import DistContext


def peer_cap_from_env() -> int:
    """``DTFS_PEER_COMM``: 0 / unset = RCCL only; 1 = one-shot peer exchange for
    messages up to 64 KiB per peer; N > 1 = up to N bytes per peer."""
    v = int(os.environ.get("DTFS_PEER_COMM", "0") or 0)
    return 0 if v <= 0 else (64 << 10 if v == 1 else v)


def create_comm(ctx: DistContext, group=None, peer_cap: Optional[int] = None, peer_timeout_s: float = 5.0,
                can_access=None):
    """A new RcclComm over the ranks of ``group`` (default: the world).

    ``peer_cap`` > 0 (default: ``peer_cap_from_env()``) also sets up the
    one-shot peer exchange (csrc/kernels/peer.hip): messages of at most that
    many bytes per peer then go through IPC-mapped mailboxes in one kernel
    instead of RCCL (latency-bound score gathers).

    Collective: every rank of the group must call it, in the same order."""
    h = hip()
    dev = ctx.device.index if ctx.device.index is not None else torch.cuda.current_device()
    cap = peer_cap_from_env() if peer_cap is None else int(peer_cap)
    if not (ctx.world > 1 and dist.is_initialized()):
        c = h.RcclComm(h.rccl_unique_id(), 1, 0, dev)
        if cap > 0:
            c.peer_enable([c.peer_prepare(cap)], peer_timeout_s)
        return c
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    obj = [h.rccl_unique_id() if rank == 0 else None]
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast_object_list(obj, src=src, group=group)
    c = h.RcclComm(obj[0], world, rank, dev)
    if cap > 0:
        enable_peer(c, cap, group, peer_timeout_s, can_access=can_access)
    return c


def enable_peer(comm, cap: int, group=None, timeout_s: float = 5.0, can_access=None) -> bool:
    """Collective: export every rank's mailbox, exchange the IPC handles over
    torch.distributed, map them. After it, every rank's exchanges of at most
    ``cap`` bytes per peer run as one peer.hip kernel.

    The kernel stores into every peer's memory directly, so it needs peer
    access between EVERY pair of devices: each rank checks
    ``hipDeviceCanAccessPeer`` to every other rank's device (``can_access``:
    a test hook with the same signature) and the ranks agree; if any pair
    cannot, no rank enables it and every exchange stays on RCCL (returns
    False)."""
    import sys

    world = dist.get_world_size(group)
    dev = torch.cuda.current_device()
    devs = [None] * world
    dist.all_gather_object(devs, dev, group=group)
    check = can_access or comm.can_access_device
    ok = all(bool(check(int(d))) for d in devs)
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    if dist.get_backend(group) != "gloo":
        flag = flag.cuda()
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if not int(flag.item()):
        print(f"[native_comm] rank {dist.get_rank(group)}: a device pair has no peer access "
              f"({'here' if not ok else 'on another rank'}); exchanges stay on RCCL", file=sys.stderr, flush=True)
        return False
    mine = comm.peer_prepare(int(cap))
    handles = [None] * comm.nranks
    dist.all_gather_object(handles, mine, group=group)
    comm.peer_enable(handles, timeout_s)
    # every rank has mapped every mailbox before anyone pushes into one
    dist.barrier(group=group)
    return True


def check_comms(*comms) -> Optional[str]:
    """First asynchronous RCCL error among ``comms`` (None when healthy)."""
    for c in comms:
        if c is None:
            continue
        e = c.async_error()
        if e:
            return e
    return None

"""Bootstrap of the native RCCL communicators (csrc/comm/rccl_comm.cpp).

torch.distributed is used once, to broadcast rank 0's 128-byte ncclUniqueId;
after that the fan-out collectives are issued from C++ by the StepRunner
(reference counterpart: the per-host channel setup, DCNClient.java:118-125).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..ops import hip
from .dist import DistContext


def create_comm(ctx: DistContext, group=None):
    """A new RcclComm over the ranks of ``group`` (default: the world).

    Collective: every rank of the group must call it, in the same order."""
    h = hip()
    dev = ctx.device.index if ctx.device.index is not None else torch.cuda.current_device()
    if not (ctx.world > 1 and dist.is_initialized()):
        return h.RcclComm(h.rccl_unique_id(), 1, 0, dev)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    obj = [h.rccl_unique_id() if rank == 0 else None]
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast_object_list(obj, src=src, group=group)
    return h.RcclComm(obj[0], world, rank, dev)


def check_comms(*comms) -> Optional[str]:
    """First asynchronous RCCL error among ``comms`` (None when healthy)."""
    for c in comms:
        if c is None:
            continue
        e = c.async_error()
        if e:
            return e
    return None

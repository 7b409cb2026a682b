"""Bootstrap of the shared-memory step control (csrc/runtime/step_control.h).

Every rank of a fan-out server maps one POSIX shared-memory segment through
which the ranks agree, per step, whether a step runs and with which padding
bucket (the largest any rank needs). Rank 0 creates the segment under a random
name, publishes the name in the job's key-value store, waits until every rank
has attached and then unlinks the name (the mappings stay; nothing is left in
``/dev/shm`` if a process dies). The store, not a collective, carries the
name, so a surviving subset of ranks can build a fresh segment for a rebuilt
cluster (serving/cluster.py recovery) without the dead rank.

Reference counterpart: none - the reference's client decides every fan-out on
its own (DCNClient.java:146-164); here the ranks of one node agree on a step.
"""
from __future__ import annotations

import datetime
import os
import secrets
import time
from typing import Optional

import torch.distributed as dist


def default_store():
    """The job's TCPStore (the one ``init_process_group`` rendezvoused on)."""
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store()


def create_control(module, world: int, rank: int, store=None, prefix: str = "dtfs/ctl/0",
                   timeout_s: float = 60.0):
    """A StepControl of ``module`` (``_hip`` for a GPU live server, ``_native``
    for a CPU one) shared by ``world`` ranks. Not a collective: every rank
    calls it with the same ``prefix`` (unique per segment) and returns once
    rank 0 has seen every rank attach."""
    store = store if store is not None else default_store()
    name_key, att_key = f"{prefix}/name", f"{prefix}/attached"
    if rank == 0:
        name = f"/dtfs-ctl-{os.getpid()}-{secrets.token_hex(6)}"
        ctl = module.StepControl(name, world, 0, True)
        store.set(name_key, name)
    else:
        store.wait([name_key], datetime.timedelta(seconds=timeout_s))
        name = store.get(name_key).decode()
        ctl = module.StepControl(name, world, rank, False)
    store.add(att_key, 1)
    if rank == 0:
        deadline = time.monotonic() + timeout_s
        try:
            while store.add(att_key, 0) < world:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"step control {name}: only {store.add(att_key, 0)} of {world} ranks attached")
                time.sleep(0.002)
        finally:
            ctl.unlink()  # every rank mapped it (or we give up): drop the name
    return ctl


def control_for_job(module, ctx, tag: str = "serve") -> Optional[object]:
    """The step control of a multi-rank job (None for one rank)."""
    if not (ctx.world > 1 and dist.is_initialized()):
        return None
    return create_control(module, ctx.world, ctx.rank, prefix=f"dtfs/ctl/{tag}")

"""Process-group bootstrap and the candidate splitter.

One process per GPU, launched by ``torch.distributed.run`` (or ``mp.spawn`` in
tests). On ROCm the ``nccl`` backend IS RCCL, so every collective below rides
xGMI between the GPUs of a node; on a CPU-only box the same code runs over
``gloo`` (that is how the distributed paths are tested without a GPU).
This replaces the reference's per-host gRPC channels (reference
DCNClient.java:118-135): connection setup is ``init_process_group``, teardown
is ``destroy_process_group`` (the reference never calls ``shutdown()``).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_distributed(self) -> bool:
        return self.world > 1 and dist.is_initialized()


def init_from_env(device: str = "auto", backend: Optional[str] = None, timeout_s: float = 300.0) -> DistContext:
    """Initialise from torchrun env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    Single process (no WORLD_SIZE or WORLD_SIZE=1) needs no process group."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if os.environ.get("DTFS_SHARE_GPU") == "1" and world > 1:
        # rehearsal of an N-rank job on fewer GPUs (a 1-GPU box): RCCL refuses
        # two ranks on one device of one host, so every rank claims its own
        # host id and the ranks talk over RCCL's socket transport instead of
        # xGMI - same communicators, collectives and step protocol
        os.environ["NCCL_HOSTID"] = f"dtfs-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    use_cuda = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_cuda:
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        # threads + pinned arenas on the GPU's socket (utils/affinity.py),
        # before the process group / live server create their threads
        from ..utils.affinity import place_rank

        place_rank(dev)
    else:
        dev = torch.device("cpu")
    be = backend or ("nccl" if use_cuda else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistContext(rank=rank, world=world, local_rank=local, device=dev, backend=be if world > 1 else "none")


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()


def split_rows(n: int, parts: int) -> List[Tuple[int, int]]:
    """Row-boundary split of n candidates into `parts` contiguous (start, size).

    The first n % parts shards get ceil(n/parts) rows, the rest floor(n/parts).
    Fixes the reference's partitionList, which splits the FLATTENED id list
    (n*43 elements) and so hands shards a row count that does not match the
    elements it sends when n*43 % parts != 0 (reference DCNClient.java:46-55,
    97)."""
    if parts <= 0:
        raise ValueError("parts must be >= 1")
    base, rem = divmod(n, parts)
    out, s = [], 0
    for i in range(parts):
        k = base + (1 if i < rem else 0)
        out.append((s, k))
        s += k
    return out


def reference_partition(items: list, parts: int) -> List[list]:
    """The reference's flat-index partitionList (kept only to document/test the bug)."""
    n = len(items)
    rng = n // parts
    out = [items[i * rng:(i + 1) * rng] for i in range(parts - 1)]
    out.append(items[(parts - 1) * rng:])
    return out

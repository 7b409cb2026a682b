"""NUMA placement of a rank: threads and pinned request arenas on the socket
its GPU hangs off (csrc/runtime/numa.h).

On an 8-GPU MI355X node four GPUs sit behind each CPU socket. A rank whose
pinned arenas - the buffers every step's H2D copy reads, most of the DeepFM
step period - or whose serving threads (submitters, launcher, completer,
decode pool) land on the far socket pays the inter-socket link on every copy
and every arena write. :func:`place_rank` runs inside the rank (not through a
launcher wrapper): the GPU's PCI bus id -> its NUMA node (sysfs) -> every
thread of the process bound to that node's CPUs (threads created later
inherit) -> the thread's memory policy prefers the node; the live server then
allocates its arenas with :func:`alloc_pinned_arena` (pages placed on the node
before ``hipHostRegister``). ``DTFS_NUMA=0`` turns it off.

The reference has no host placement (a Java client against remote hosts,
DCNClient.java:118-125).
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import torch

log = logging.getLogger(__name__)

_placement: dict = {"node": -1}


def current_node() -> int:
    """The NUMA node this rank placed itself on (-1: none)."""
    return int(_placement.get("node", -1))


def placement() -> dict:
    return dict(_placement)


def place_on_node(node: int) -> dict:
    """Bind every thread of the process to ``node``'s CPUs (those this process
    may use) and prefer ``node`` for this thread's future allocations."""
    from ..ops import native

    n = native()
    allowed = os.sched_getaffinity(0)
    cpus = [c for c in n.numa_node_cpus(int(node)) if c in allowed]
    info = {"node": int(node), "cpus": len(cpus), "threads_bound": 0, "numa_nodes": int(n.numa_node_count())}
    if not cpus:  # a cpuset that excludes the node: leave the threads where they are
        info["note"] = "no allowed CPU on the node"
        return info
    info["threads_bound"] = int(n.bind_process_cpus(cpus))
    info["mempolicy"] = bool(n.prefer_numa_node(int(node)))
    _placement.clear()
    _placement.update(info)
    return info


def place_rank(device: torch.device) -> dict:
    """Place this rank on its GPU's NUMA node (no-op on CPU devices, on
    single-node machines, when the platform reports no node, or DTFS_NUMA=0)."""
    if device.type != "cuda" or os.environ.get("DTFS_NUMA", "1") == "0":
        return {"node": -1}
    from ..ops import hip, native

    bus = hip().pci_bus_id(int(device.index or 0))
    node = int(native().pci_numa_node(bus)) if bus else -1
    if node < 0 or native().numa_node_count() < 2:
        _placement.update(node=-1, pci_bus_id=bus, numa_nodes=int(native().numa_node_count()))
        return placement()
    info = place_on_node(node)
    info["pci_bus_id"] = bus
    _placement.update(info)
    log.info("rank on %s: NUMA node %d, %d CPUs, %d threads bound", bus, node, info["cpus"], info["threads_bound"])
    return info


def alloc_pinned_arena(nbytes: int, node: Optional[int] = None) -> torch.Tensor:
    """A pinned uint8 host buffer for a GPU live server: on this rank's NUMA
    node when it has one (pages placed first, then hipHostRegister), else
    torch's pinned allocator."""
    node = current_node() if node is None else node
    if node >= 0:
        from ..ops import hip

        return hip().alloc_pinned_on_node(int(nbytes), int(node))
    return torch.zeros(int(nbytes), dtype=torch.uint8, pin_memory=True)

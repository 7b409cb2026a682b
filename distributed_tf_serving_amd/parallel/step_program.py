"""Programmed steps: a forward that interleaves kernels with collectives, as a
short op list over two device lanes.

The candidate fan-out (parallel/fanout.py) has a fixed shape - exchange rows,
run the forward graph, exchange scores - so the native StepRunner has a
dedicated ``launch_fanout``. Embedding model parallelism (DLRM with sharded
tables, SURVEY.md §2.5 C3, BASELINE config 4) interleaves them instead:

    aux lane      route ids -> ids all-to-all -> owner-side gather -> embeddings all-to-all
    compute lane  bottom MLP (overlaps the exchange)          -> interaction + top MLP + head

A model describes one step as a list of :class:`Kernels` / :class:`Coll` /
:class:`Sync` ops whose tensors are static (allocated once per bucket and
slot). The same list runs three ways:

* :func:`run_eager` - in order, collectives through torch.distributed (CPU /
  gloo tests, the eager GPU fallback);
* :func:`capture_native` - every ``Kernels`` op captured into its own HIP
  graph (one memory pool and capture stream per lane), the whole list handed
  to ``StepRunner.launch_program`` (csrc/runtime/step_runner.h) with native
  RCCL communicators: the live server's step, no Python per step.

Lanes meet only through ``Sync`` record / wait pairs on per-slot events; the
step is done when the compute lane is, and the native side rejects a program
whose aux-lane work is not joined into the compute lane.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Union

import torch
import torch.distributed as dist

COMPUTE, AUX = 0, 1


@dataclass
class Kernels:
    lane: int
    fn: Callable[[], None]
    name: str = ""


@dataclass
class Coll:
    kind: str  # "alltoall" | "allgather" | "reduce_scatter" (bf16 sum)
    lane: int
    send: torch.Tensor
    recv: torch.Tensor


@dataclass
class Sync:
    kind: str  # "record" | "wait" | "wait_prev" (the event of the previous step, any slot)
    lane: int
    event: int


Op = Union[Kernels, Coll, Sync]


def validate(ops: Sequence[Op]) -> None:
    """Python mirror of StepProgram::validate (CPU tests run no native code)."""
    aux_ops, joined = 0, 0
    covers: Dict[int, int] = {}
    for o in ops:
        if isinstance(o, Sync):
            if not 0 <= o.event < 8:
                raise ValueError("event index out of range")
            if o.kind == "record":
                covers[o.event] = aux_ops if o.lane == AUX else 0
            elif o.kind == "wait":
                if o.event not in covers:
                    raise ValueError("event waited before it is recorded")
                if o.lane == COMPUTE:
                    joined = max(joined, covers[o.event])
            elif o.kind != "wait_prev":
                raise ValueError(f"unknown sync {o.kind!r}")
        elif o.lane == AUX:
            aux_ops += 1
    if joined < aux_ops:
        raise ValueError("aux-lane work is not joined into the compute lane")


def _wire(t: torch.Tensor, group) -> torch.Tensor:
    # gloo has no bf16 collectives: exchange fp32 copies
    if t.dtype == torch.bfloat16 and dist.is_initialized() and dist.get_backend(group) == "gloo":
        return t.float()
    return t


def _collective(c: Coll, group) -> None:
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:  # every collective of one rank is a copy
        c.recv.view(-1).copy_(c.send.reshape(-1))
        return
    gloo = dist.get_backend(group) == "gloo"
    send, out = _wire(c.send, group), _wire(c.recv, group)  # out is c.recv unless it needed an fp32 copy
    if c.kind == "alltoall":
        dist.all_to_all_single(out.view(-1), send.reshape(-1), group=group)
    elif c.kind == "allgather":
        if gloo:
            dist.all_gather(list(out.view(world, -1).unbind(0)), send.reshape(-1), group=group)
        else:
            dist.all_gather_into_tensor(out.view(-1), send.reshape(-1), group=group)
    elif c.kind == "reduce_scatter":
        if gloo:  # no reduce_scatter on gloo: all-reduce fp32 and keep this rank's slice
            full = send.float().reshape(world, -1).clone()
            dist.all_reduce(full, group=group)
            out = full[dist.get_rank(group)]
        else:
            dist.reduce_scatter_tensor(out.view(-1), send.reshape(-1), group=group)
    else:
        raise ValueError(f"unknown collective {c.kind!r}")
    if out is not c.recv:
        c.recv.view(-1).copy_(out.reshape(-1))


def run_eager(ops: Sequence[Op], group=None) -> None:
    """Run a program in list order on the current stream (a valid schedule of
    the two lanes); collectives through torch.distributed."""
    for o in ops:
        if isinstance(o, Kernels):
            o.fn()
        elif isinstance(o, Coll):
            _collective(o, group)


@dataclass
class NativeProgram:
    """A captured program: the dict StepRunner.launch_program / the live
    server take, plus the graphs and sequences it points into."""

    spec: dict
    graphs: List[object]
    seqs: List[object]
    comms: List[object]


def capture_native(ops: Sequence[Op], h2d_dst: torch.Tensor, comm, pools: Dict[int, object],
                   streams: Dict[int, "torch.cuda.Stream"], direct: bool = True,
                   h2d_lane: int = AUX) -> NativeProgram:
    """Capture every ``Kernels`` op into its own HIP graph (lane pools /
    capture streams persist across a slot's ops so a lane's buffers are never
    shared with the other lane) and build the native program description."""
    from ..ops import hip

    validate(ops)
    h = hip()
    graphs, seqs, out = [], [], []
    for o in ops:
        if isinstance(o, Kernels):
            st = streams[o.lane]
            st.wait_stream(torch.cuda.current_stream(h2d_dst.device))
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g, pool=pools[o.lane], stream=st):
                o.fn()
            g.instantiate()
            graphs.append(g)
            seq = None
            if direct:
                try:
                    seq = h.KernelSequence(g.raw_cuda_graph())
                except RuntimeError:  # a node the sequence cannot replay: launch the graph
                    seq = None
            seqs.append(seq)
            out.append({"kind": "kernels", "lane": o.lane, "seq": seq, "graph_exec": g.raw_cuda_graph_exec()})
        elif isinstance(o, Coll):
            out.append({"kind": o.kind, "lane": o.lane, "comm": comm, "send": o.send, "recv": o.recv})
        else:
            out.append({"kind": o.kind, "lane": o.lane, "event": o.event})
    spec = {"h2d_dst": h2d_dst, "h2d_lane": h2d_lane, "ops": out}
    return NativeProgram(spec=spec, graphs=graphs, seqs=seqs, comms=[comm])

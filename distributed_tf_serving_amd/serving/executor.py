"""ShardExecutor: one device's model runner over packed request rows.

Per batch-size bucket (TF-Serving's ``allowed_batch_sizes``) and per pipeline
slot it owns a static device input buffer, and on a GPU it captures the whole
forward (gather -> interaction -> MLP GEMMs -> head) into a HIP graph once, so
a batch costs one graph launch instead of 6-10 kernel launches from Python.
Slots let the next batch's H2D/collectives overlap the current batch's compute
without the two sharing static buffers.
"""
from __future__ import annotations

import bisect
import threading
from typing import Dict, Optional, Sequence, Tuple

import torch

from .packing import PackedLayout


class ShardExecutor:
    def __init__(self, model: torch.nn.Module, layout: PackedLayout, buckets: Sequence[int],
                 device: torch.device, use_graphs: bool = True, slots: int = 2, warmup: int = 2):
        self.model = model
        self.layout = layout
        self.buckets = sorted(set(int(b) for b in buckets))
        self.device = torch.device(device)
        self.is_cuda = self.device.type == "cuda"
        # a forward that issues collectives itself (sharded DLRM tables) runs eagerly
        self.use_graphs = bool(use_graphs and self.is_cuda and not getattr(model, "has_collectives", False))
        self.slots = max(1, int(slots))
        self.warmup = warmup
        self._inp: Dict[Tuple[int, int], torch.Tensor] = {}
        self._out: Dict[Tuple[int, int], torch.Tensor] = {}
        self._graphs: Dict[Tuple[int, int], "torch.cuda.CUDAGraph"] = {}
        self._pools = {}
        self._lock = threading.Lock()

    # -- buckets -------------------------------------------------------------
    @property
    def max_rows(self) -> int:
        return self.buckets[-1]

    def bucket_for(self, n: int) -> int:
        i = bisect.bisect_left(self.buckets, n)
        if i == len(self.buckets):
            raise ValueError(f"{n} rows exceed the largest bucket {self.buckets[-1]}")
        return self.buckets[i]

    # -- buffers ---------------------------------------------------------------
    def input_buffer(self, B: int, slot: int = 0) -> torch.Tensor:
        key = (B, slot)
        buf = self._inp.get(key)
        if buf is None:
            buf = self.layout.alloc(B, device=self.device)
            self._inp[key] = buf
        return buf

    def _forward(self, buf: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        if out is None:
            return self.model(self.layout.ids(buf), self.layout.wts(buf))
        return self.model(self.layout.ids(buf), self.layout.wts(buf), out=out)

    def prepare(self, B: int, slot: int = 0) -> None:
        """Allocate (and on GPU capture) bucket B for a slot ahead of traffic."""
        key = (B, slot)
        if key in self._out:
            return
        with self._lock:
            if key in self._out:
                return
            buf = self.input_buffer(B, slot)
            if not self.use_graphs:
                self._out[key] = None
                return
            dev = self.device
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(self.warmup):
                    self._forward(buf)
            torch.cuda.current_stream(dev).wait_stream(side)
            pool = self._pools.get(slot)
            if pool is None:
                pool = self._pools[slot] = torch.cuda.graph_pool_handle()
            # keep the hipGraph_t: the native loop replays its nodes as direct
            # launches (runtime/kernel_seq.cpp); replay() uses the instantiated exec
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g, pool=pool):
                out = self._forward(buf)
            g.instantiate()
            self._graphs[key] = g
            self._out[key] = out

    def prepare_all(self) -> None:
        for B in self.buckets:
            for s in range(self.slots):
                self.prepare(B, s)

    # -- execution -------------------------------------------------------------
    def run(self, B: int, slot: int = 0, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Run bucket B on its static input buffer (or ``buf``); returns CTR [B] fp32.

        On GPU the returned tensor is the graph's static output: consume it (copy
        or enqueue dependent work) before the same (bucket, slot) runs again."""
        if buf is not None and buf is not self._inp.get((B, slot)):
            if self.use_graphs:
                self.input_buffer(B, slot).copy_(buf[:B], non_blocking=True)
            else:
                return self._forward(buf[:B])
        if not self.use_graphs:
            return self._forward(self.input_buffer(B, slot))
        self.prepare(B, slot)
        self._graphs[(B, slot)].replay()
        return self._out[(B, slot)]

    def run_rows(self, ids: torch.Tensor, wts: torch.Tensor) -> torch.Tensor:
        """Convenience (tests, CPU backend): run unpacked ids/wts of any row count."""
        n = ids.shape[0]
        if not self.use_graphs:
            return self.model(ids.to(self.device), wts.to(self.device))[:n]
        outs = []
        for s in range(0, n, self.max_rows):
            e = min(n, s + self.max_rows)
            B = self.bucket_for(e - s)
            buf = self.input_buffer(B, 0)
            buf.zero_()
            self.layout.ids(buf)[: e - s].copy_(ids[s:e])
            self.layout.wts(buf)[: e - s].copy_(wts[s:e])
            outs.append(self.run(B, 0)[: e - s].clone())
        return torch.cat(outs)

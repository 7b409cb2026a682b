"""Host-side step pipeline for one rank: decode -> H2D -> forward -> D2H -> encode.

Stages and where they run::

    produce(k, slot)   request decode into host_in(B, slot)   host pool thread
    engine.launch()    H2D [SDMA] -> collectives -> graph       GPU queues
    handle.wait()      scores landed in host_out(B, slot)      main thread
    consume(k, ctx)    response encode                          host thread

Buffers cycle over S slots. Step k is enqueued as soon as its decode is done,
so its H2D starts while earlier steps compute; the host keeps ``depth`` steps
queued on the GPU. Slot reuse rules (S >= depth + 1):

* decode(k) writes host_in[k % S]: step k - S must have completed (its H2D read
  that buffer) - guaranteed because decode(k) starts after finish(k - depth).
* launch(k) D2H-writes host_out[k % S]: consume(k - S) must have finished.
"""
from __future__ import annotations

import concurrent.futures as cf
import time
from typing import Any, Callable, Dict, List, Optional


class StepPipeline:
    def __init__(self, engine, B: int, slots: int = 3, depth: int = 2,
                 produce: Callable[[int, int], Any] = None, consume: Callable[[int, Any, Any], Any] = None,
                 launch: Optional[Callable[[int, int, Any], Any]] = None):
        """``launch(k, slot, ctx)`` overrides ``engine.launch(B, slot)`` (e.g. to
        pass an arena and its used byte count)."""
        if slots < depth + 1:
            raise ValueError("need slots >= depth + 1")
        self.eng, self.B, self.S, self.depth = engine, B, slots, depth
        self.produce, self.consume = produce, consume
        self.launch_fn = launch
        self.dec_pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="dtfs-decode")
        self.enc_pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="dtfs-encode")
        self.latencies: List[float] = []
        self.phase = {"decode_wait": 0.0, "enc_wait": 0.0, "launch": 0.0, "gpu_wait": 0.0}

    def reset_stats(self):
        self.latencies.clear()
        for k in self.phase:
            self.phase[k] = 0.0

    def run(self, n_steps: int, record: bool = True) -> None:
        S, depth = self.S, self.depth
        t_start: Dict[int, float] = {}
        dec: Dict[int, cf.Future] = {}
        enc: Dict[int, cf.Future] = {}
        handles: Dict[int, Any] = {}
        ctxs: Dict[int, Any] = {}

        def start_decode(j: int) -> None:
            t_start[j] = time.perf_counter()
            dec[j] = self.dec_pool.submit(self.produce, j, j % S)

        def finish(j: int) -> None:
            t = time.perf_counter()
            scores = handles.pop(j).wait()
            now = time.perf_counter()
            self.phase["gpu_wait"] += now - t
            lat = now - t_start.pop(j)
            if record:
                self.latencies.append(lat)
            enc[j] = self.enc_pool.submit(self.consume, j, ctxs.pop(j), scores)

        for j in range(min(depth, n_steps)):
            start_decode(j)
        for k in range(n_steps):
            t1 = time.perf_counter()
            ctxs[k] = dec.pop(k).result()
            t2 = time.perf_counter()
            f = enc.pop(k - S, None)
            if f is not None:
                f.result()
            t3 = time.perf_counter()
            if self.launch_fn is not None:
                handles[k] = self.launch_fn(k, k % S, ctxs[k])
            else:
                handles[k] = self.eng.launch(self.B, k % S)
            t4 = time.perf_counter()
            self.phase["decode_wait"] += t2 - t1
            self.phase["enc_wait"] += t3 - t2
            self.phase["launch"] += t4 - t3
            if k - depth + 1 >= 0:
                finish(k - depth + 1)
            if k + depth < n_steps:
                start_decode(k + depth)
        for j in sorted(handles):
            finish(j)
        for f in enc.values():
            f.result()

    def close(self) -> None:
        self.dec_pool.shutdown(wait=True)
        self.enc_pool.shutdown(wait=True)

"""Server-side dynamic batching (the TF-Serving feature the reference relies on,
reference README.md:5,9), re-built around a GPU shard.

Concurrent Predict calls become :class:`WorkItem`\\ s. The native
``DynamicBatcher`` (csrc/runtime/batcher.cpp) coalesces them until
``max_batch_rows`` or ``batch_timeout_us``; one worker thread per servable then

1. picks the smallest bucket >= the batch's rows (``allowed_batch_sizes``: the
   shapes the HIP graphs were captured for),
2. has every item decode itself straight into that bucket's pinned packed-row
   buffer (no intermediate copies),
3. launches the step on the GPU and, while it runs, already forms and launches
   the next batch (up to ``depth`` steps in flight over ``slots`` buffers),
4. splits the returned CTR vector back into per-request futures.

Requests whose deadline passed while queued fail with DEADLINE_EXCEEDED
instead of consuming GPU time; a full queue rejects with RESOURCE_EXHAUSTED.
"""
from __future__ import annotations

import collections
import concurrent.futures as cf
import itertools
import logging
import threading
from dataclasses import dataclass
from typing import Callable, Deque, Dict, List, Optional

import torch

from ..ops import native
from .errors import Code, ServingError

log = logging.getLogger(__name__)


class _AfterLaunchNotice(Exception):
    """A launch that failed after ``on_launch`` told the follower ranks."""


@dataclass
class WorkItem:
    rows: int
    fill: Callable[[torch.Tensor, torch.Tensor], None]  # (ids_rows_view, wts_rows_view) -> None
    future: cf.Future


class BatchingScheduler:
    def __init__(self, engine, max_batch_rows: int = 8192, batch_timeout_us: int = 200,
                 max_queued_rows: int = 1 << 22, depth: int = 2, name: str = "model",
                 fanout_world: int = 1, on_launch: Optional[Callable[[int, int], None]] = None,
                 max_request_rows: int = 1 << 18, on_broken: Optional[Callable[[str], None]] = None):
        """``fanout_world`` > 1: this is the front door of a scatter fan-out
        (parallel/fanout.py): a step of bucket B carries up to world x B rows,
        split across the ranks. ``on_launch(B, slot)`` runs right before each
        step is launched (serving/cluster.py tells the follower ranks)."""
        self.eng = engine
        self.ex = engine.ex
        self.name = name
        # a failed multi-rank step (launch error after the followers were told,
        # a step timeout, a communicator error) leaves the ranks' collective
        # sequences out of step: the scheduler is then BROKEN - every queued and
        # later request fails UNAVAILABLE and on_broken(reason) tears down
        self.on_broken = on_broken
        self.broken: Optional[str] = None
        self.layout = engine.layout
        self.world = max(1, int(fanout_world))
        self.on_launch = on_launch
        self.eager_when_idle = True
        self.max_rows = min(int(max_batch_rows), self.ex.max_rows) * self.world
        # a request's declared rows are checked before anything is allocated for
        # it (TF fill semantics let a ~100-byte request declare any shape)
        self.max_request_rows = min(int(max_request_rows), int(max_queued_rows))
        self.depth = max(1, min(depth, self.ex.slots - 1)) if self.ex.slots > 1 else 1
        self.batcher = native().DynamicBatcher(self.max_rows, int(batch_timeout_us), int(max_queued_rows))
        self._items: Dict[int, WorkItem] = {}
        self._lock = threading.Lock()
        self._tickets = itertools.count(1)
        self._slot = 0
        self.steps = 0
        self.rows_served = 0
        self._worker = threading.Thread(target=self._loop, name=f"dtfs-batch-{name}", daemon=True)
        self._worker.start()

    # -- client side -------------------------------------------------------------
    def submit(self, rows: int, fill, deadline_us: int = 0) -> cf.Future:
        fut: cf.Future = cf.Future()
        if self.broken is not None:
            fut.set_exception(ServingError(Code.UNAVAILABLE, f"server unavailable: {self.broken}"))
            return fut
        if rows <= 0:
            fut.set_result(torch.empty(0))
            return fut
        if rows > self.max_request_rows:
            fut.set_exception(ServingError(
                Code.INVALID_ARGUMENT, f"request has {rows} rows; this server accepts at most {self.max_request_rows}"))
            return fut
        if rows > self.max_rows:
            # larger than one GPU batch: split into row chunks, join in order
            return self._submit_split(rows, fill, deadline_us)
        t = next(self._tickets)
        with self._lock:
            self._items[t] = WorkItem(rows, fill, fut)
        if not self.batcher.submit(t, rows, deadline_us):
            with self._lock:
                self._items.pop(t, None)
            code = Code.UNAVAILABLE if self.batcher.closed else Code.RESOURCE_EXHAUSTED
            fut.set_exception(ServingError(code, "batching queue is full" if code == Code.RESOURCE_EXHAUSTED
                                           else "server is shutting down"))
        return fut

    def _submit_split(self, rows, fill, deadline_us) -> cf.Future:
        # decode the whole request once into a staging buffer, then feed chunks
        F = self.layout.fields
        ids = torch.empty(rows, F, dtype=torch.int64)
        wts = torch.empty(rows, F, dtype=torch.float32)
        fill(ids, wts)
        parts = []
        for s in range(0, rows, self.max_rows):
            e = min(rows, s + self.max_rows)

            def f(iv, wv, s=s, e=e):
                iv.copy_(ids[s:e])
                wv.copy_(wts[s:e])

            parts.append(self.submit(e - s, f, deadline_us))
        out: cf.Future = cf.Future()

        def done(_):
            if all(p.done() for p in parts) and not out.done():
                try:
                    out.set_result(torch.cat([p.result() for p in parts]))
                except Exception as e:  # noqa: BLE001
                    out.set_exception(e)

        for p in parts:
            p.add_done_callback(done)
        return out

    # -- worker ------------------------------------------------------------------
    def mark_broken(self, reason: str) -> None:
        """Stop serving (idempotent): queued and later requests fail UNAVAILABLE."""
        if self.broken is not None:
            return
        self.broken = reason
        log.error("batching scheduler of %s broken: %s", self.name, reason)
        self.batcher.close()
        if self.on_broken is not None:
            try:
                self.on_broken(reason)
            except Exception:  # noqa: BLE001 - best effort teardown
                log.exception("on_broken failed")

    def _fail_items(self, items, reason: str) -> None:
        for it in items:
            w = self._pop(it.ticket)
            if w is not None and not w.future.done():
                w.future.set_exception(ServingError(Code.UNAVAILABLE, f"server unavailable: {reason}"))

    def _loop(self) -> None:
        inflight: Deque = collections.deque()
        while True:
            if self.broken is not None:
                # drain: everything still queued fails, in-flight steps get a short grace
                while inflight:
                    self._complete(inflight.popleft())
                batch = self.batcher.next_batch(0, True)
                self._fail_items(batch.items, self.broken)
                self._fail_items(batch.expired, self.broken)
                if batch.closed and not batch.items:
                    with self._lock:
                        left = list(self._items.values())
                        self._items.clear()
                    for w in left:
                        if not w.future.done():
                            w.future.set_exception(ServingError(Code.UNAVAILABLE, f"server unavailable: {self.broken}"))
                    break
                continue
            # idle device: dispatch whatever is queued right away (latency);
            # steps in flight: accumulate up to the batch timeout (throughput)
            batch = self.batcher.next_batch(0 if inflight else 50_000, self.eager_when_idle and not inflight)
            for it in batch.expired:
                w = self._pop(it.ticket)
                if w is not None:
                    w.future.set_exception(ServingError(Code.DEADLINE_EXCEEDED, "request deadline exceeded while queued"))
            if batch.items:
                try:
                    inflight.append(self._launch(batch))
                except _AfterLaunchNotice as e:
                    # the followers already joined this step: the ranks are out of step
                    self._fail_items(batch.items, f"step launch failed: {e.__cause__}")
                    self.mark_broken(f"step launch failed after the followers were told: {e.__cause__}")
                    continue
                except Exception as e:  # noqa: BLE001 - fail the batch, keep serving
                    log.exception("batch launch failed")
                    for it in batch.items:
                        w = self._pop(it.ticket)
                        if w is not None and not w.future.done():
                            w.future.set_exception(ServingError(Code.INTERNAL, f"batch failed: {e}"))
            if inflight and (len(inflight) >= self.depth or not batch.items):
                self._complete(inflight.popleft())
            if batch.closed and not batch.items and not inflight:
                break

    def _pop(self, ticket: int) -> Optional[WorkItem]:
        with self._lock:
            return self._items.pop(ticket, None)

    def _launch(self, batch):
        rows = batch.rows
        B = self.ex.bucket_for(-(-rows // self.world))  # rows per GPU
        slot = self._slot
        self._slot = (self._slot + 1) % self.ex.slots
        buf = self.eng.host_in(B, slot)
        ids_v, wts_v = self.layout.ids(buf), self.layout.wts(buf)
        plan: List = []
        off = 0
        for it in batch.items:
            w = self._pop(it.ticket)
            if w is None:
                continue
            try:
                w.fill(ids_v[off:off + w.rows], wts_v[off:off + w.rows])
            except Exception as e:  # noqa: BLE001 - malformed request: fail it alone
                ids_v[off:off + w.rows].zero_()
                wts_v[off:off + w.rows].zero_()
                err = e if isinstance(e, ServingError) else ServingError(Code.INVALID_ARGUMENT, str(e))
                w.future.set_exception(err)
                off += w.rows
                continue
            plan.append((w, off))
            off += w.rows
        total = B * self.world
        if off < total:  # padding rows: valid ids, zero weights (their scores are dropped)
            ids_v[off:total].zero_()
            wts_v[off:total].zero_()
        if self.on_launch is not None:
            try:
                self.on_launch(B, slot)
            except Exception as e:  # the control channel is gone: nobody can join this step
                for w, _ in plan:
                    w.future.set_exception(ServingError(Code.UNAVAILABLE, f"step control failed: {e}"))
                self.mark_broken(f"step control channel failed: {e}")
                raise _AfterLaunchNotice() from e
            try:
                handle = self.eng.launch(B, slot)
            except Exception as e:
                for w, _ in plan:
                    w.future.set_exception(ServingError(Code.UNAVAILABLE, f"step launch failed: {e}"))
                raise _AfterLaunchNotice() from e
        else:
            handle = self.eng.launch(B, slot)
        return handle, plan, off

    def _complete(self, entry) -> None:
        handle, plan, rows = entry
        if self.broken is not None and handle.timeout_s is not None:
            handle.timeout_s = min(handle.timeout_s, 0.5)
        try:
            scores = handle.wait()
        except Exception as e:  # noqa: BLE001 - a step that never finishes or failed
            for w, _ in plan:
                if not w.future.done():
                    w.future.set_exception(ServingError(Code.UNAVAILABLE, f"server unavailable: {e}"))
            self.mark_broken(str(e))
            return
        self.steps += 1
        self.rows_served += rows
        for w, off in plan:
            if not w.future.done():
                w.future.set_result(scores[off:off + w.rows].clone())

    def stats(self) -> dict:
        st = self.batcher.stats()
        return {"submitted": st.submitted, "rejected": st.rejected, "batches": st.batches,
                "batched_rows": st.batched_rows, "expired": st.expired, "full_batches": st.full_batches,
                "timeout_batches": st.timeout_batches, "steps": self.steps, "rows_served": self.rows_served}

    def close(self) -> None:
        self.batcher.close()
        self._worker.join(timeout=30)

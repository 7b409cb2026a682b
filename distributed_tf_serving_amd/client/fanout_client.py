"""Async fan-out client: split one request's candidates across N backends,
dispatch in parallel, gather the CTR scores (reference DCNClient.processARequest,
DCNClient.java:137-203).

Differences from the reference, each a documented fix:

* candidates are split on ROW boundaries (``split_rows``), not on the flat
  id list, so every shard request is well-formed for any N;
* the request spec is immutable (the reference shares one protobuf Builder
  across 16 threads);
* sorting returns the permutation too, so ranked scores keep their candidate;
* completion-order gather uses ``as_completed`` instead of a busy poll;
* failures propagate as exceptions with the shard index (no silent return).

``full_async=True`` (mode A, the reference default) joins shards in shard order;
``False`` (mode B) concatenates in completion order, like the reference's
polling loop (DCNClient.java:165-193).
"""
from __future__ import annotations

import concurrent.futures as cf
import threading
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops import native
from ..parallel.dist import split_rows
from ..wire import schema as pb
from .backends import Backend


@dataclass(frozen=True)
class RequestSpec:
    model_name: str = "DCN"
    signature_name: str = "serving_default"
    version: Optional[int] = None
    ids_key: str = "feat_ids"
    wts_key: str = "feat_wts"
    output_key: str = "prediction_node"
    raw: bool = False  # tensor_content encoding instead of int64_val / float_val


@dataclass
class FanoutResult:
    scores: torch.Tensor                       # per candidate, candidate order (mode A) or completion order (B)
    sorted_scores: Optional[torch.Tensor] = None
    order: Optional[torch.Tensor] = None       # candidate index of each sorted score
    shard_order: Optional[List[int]] = None    # order shards were concatenated in


class ShardError(RuntimeError):
    def __init__(self, shard: int, backend: str, cause: BaseException):
        super().__init__(f"shard {shard} ({backend}) failed: {cause!r}")
        self.shard, self.backend, self.cause = shard, backend, cause


class FanoutClient:
    def __init__(self, backends: Sequence[Backend], spec: RequestSpec = RequestSpec(), pool_threads: int = 16,
                 full_async: bool = True, sort_scores: bool = True, timeout_s: Optional[float] = None,
                 executor: Optional[cf.Executor] = None, failover: bool = False, cooldown_s: float = 5.0):
        """``failover``: a shard whose backend fails (error or ``timeout_s``)
        is re-split over the backends still healthy and retried, and the failed
        backend is skipped by new requests for ``cooldown_s`` (degraded mode;
        the reference abandons the request, DCNClient.java:185-188)."""
        if not backends:
            raise ValueError("need at least one backend")
        self.backends = list(backends)
        self.spec = spec
        self.full_async = full_async
        self.sort_scores = sort_scores
        self.timeout_s = timeout_s
        self.failover = failover
        self.cooldown_s = cooldown_s
        self._down_until = [0.0] * len(self.backends)
        self._health_lock = threading.Lock()
        self.failovers = 0
        self._own_pool = executor is None
        self.pool = executor or cf.ThreadPoolExecutor(max_workers=pool_threads, thread_name_prefix="dtfs-fanout")
        self.nat = native()

    # -- health -----------------------------------------------------------------
    def healthy(self) -> List[int]:
        """Backends not in cool-down (all of them if every one is down)."""
        now = time.monotonic()
        with self._health_lock:
            alive = [i for i, t in enumerate(self._down_until) if t <= now]
        return alive or list(range(len(self.backends)))

    def mark_down(self, i: int) -> None:
        with self._health_lock:
            self._down_until[i] = time.monotonic() + self.cooldown_s

    # -- encoding -------------------------------------------------------------
    def encode(self, ids: torch.Tensor, wts: torch.Tensor) -> bytes:
        s = self.spec
        return self.nat.encode_predict_request(s.model_name, s.signature_name, s.version,
                                               [(s.ids_key, ids), (s.wts_key, wts)], s.raw)

    def decode_scores(self, data: bytes) -> torch.Tensor:
        r = pb.PredictResponse.FromString(data)
        t = r.outputs[self.spec.output_key]
        if t.tensor_content:
            return torch.from_numpy(np.frombuffer(t.tensor_content, dtype="<f4").copy())
        return torch.tensor(list(t.float_val), dtype=torch.float32)

    # -- fan-out ----------------------------------------------------------------
    def _call(self, i: int, ids: torch.Tensor, wts: torch.Tensor) -> torch.Tensor:
        be = self.backends[i]
        try:
            return self.decode_scores(be.predict(self.encode(ids, wts), self.timeout_s))
        except BaseException as e:  # noqa: BLE001
            raise ShardError(i, be.name, e) from e

    def _shard_call(self, i: int, ids: torch.Tensor, wts: torch.Tensor) -> torch.Tensor:
        try:
            return self._call(i, ids, wts)
        except ShardError:
            if not self.failover:
                raise
            self.mark_down(i)
            alive = [j for j in self.healthy() if j != i and self._down_until[j] <= time.monotonic()]
            if not alive:
                raise
            self.failovers += 1
            # degraded mode: re-split this shard over the surviving backends
            outs = []
            for j, (s, k) in zip(alive, split_rows(ids.shape[0], len(alive))):
                if k:
                    try:
                        outs.append(self._call(j, ids[s:s + k], wts[s:s + k]))
                    except ShardError:
                        self.mark_down(j)
                        raise
            return torch.cat(outs)

    def predict_async(self, ids, wts) -> cf.Future:
        """Returns a Future[FanoutResult] (CompletableFuture analogue)."""
        ids = torch.as_tensor(ids, dtype=torch.int64)
        wts = torch.as_tensor(wts, dtype=torch.float32)
        n = ids.shape[0]
        targets = self.healthy() if self.failover else list(range(len(self.backends)))
        parts = [(targets[i], s, k) for i, (s, k) in enumerate(split_rows(n, len(targets))) if k > 0]
        futs = {self.pool.submit(self._shard_call, i, ids[s:s + k], wts[s:s + k]): i for i, s, k in parts}
        out: cf.Future = cf.Future()
        if not futs:
            out.set_result(FanoutResult(scores=torch.empty(0)))
            return out
        state = {"left": len(futs), "done": []}
        lock = threading.Lock()

        def on_done(f: cf.Future):
            with lock:
                state["done"].append(futs[f])
                state["left"] -= 1
                if state["left"]:
                    return
            try:
                if self.full_async:  # mode A: shard order (candidate order)
                    order = [i for i, _, _ in parts]
                else:  # mode B: completion order
                    order = list(state["done"])
                by_idx = {futs[g]: g for g in futs}
                scores = torch.cat([by_idx[i].result() for i in order])
                res = FanoutResult(scores=scores, shard_order=order)
                if self.sort_scores:
                    res.sorted_scores, res.order = torch.sort(scores, stable=True)
                out.set_result(res)
            except BaseException as e:  # noqa: BLE001
                out.set_exception(e)

        for f in futs:
            f.add_done_callback(on_done)
        return out

    def predict(self, ids, wts) -> FanoutResult:
        return self.predict_async(ids, wts).result()

    def close(self) -> None:
        if self._own_pool:
            self.pool.shutdown(wait=True)
        for b in self.backends:
            b.close()

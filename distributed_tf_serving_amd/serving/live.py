"""Live native serving endpoint of one servable (csrc/runtime/live_server.h).

Every Predict of a GPU servable - gRPC front door, in-process clients, the
bench's native load generator - enters :meth:`LiveScheduler.predict_bytes`
(or the C++ ``submit``): the request is validated, admitted into the dynamic
batch and copied ONCE into a pinned request arena; the C++ launcher closes the
batch (``max_batch_rows`` / ``batch_timeout_us`` / device idle), the GPU
unpacks the raw request bytes inside the captured step kernels, and the C++
completer encodes each PredictResponse. No Python runs per request on the fast
path; the reference's server (TF-Serving with batching, reference README.md:5,9;
DCNClient.java:111-112 calls it) is what this replaces.

Slow paths (a request larger than one batch, Predict with message objects,
Classify / Regress over tf.Example) go through :meth:`submit`, which encodes
the rows as raw ``tensor_content`` requests of at most one batch each and
joins their scores - the same engine either way.

On a CPU servable (BASELINE config 1) the same C++ core runs with a Python
forward as its backend.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
from typing import List, Optional, Sequence

import numpy as np
import torch

from ..ops import native
from .errors import Code, ServingError

log = logging.getLogger(__name__)


from .packing import host_narrow_modulo  # noqa: E402


def _code(c: int) -> Code:
    try:
        return Code(int(c))
    except ValueError:
        return Code.UNKNOWN


class LiveScheduler:
    """The servable's batching scheduler, backed by the native live server."""

    def __init__(self, engine, serving_cfg, buckets: Optional[Sequence[int]] = None, n_arenas: Optional[int] = None,
                 depth: Optional[int] = None, control=None, step_timeout_s: float = 10.0,
                 model_name: Optional[str] = None, version: Optional[int] = None, start_paused: bool = False,
                 narrow: Optional[bool] = None, peer_timeout_s: float = 5.0, liveness_only: bool = False):
        """``control``: the job's StepControl (parallel/control.py) when the
        step has collectives (fan-out, sharded tables): every step is then
        agreed with the other ranks - launched only when some rank has work,
        at the largest bucket any rank needs (csrc/runtime/step_control.h).
        ``liveness_only``: the control only carries heartbeats and the broken
        flag - steps are this rank's own (no collectives in them) but read the
        other ranks' memory (the sharded DLRM's peer exchange), so a silent peer
        must still fail requests UNAVAILABLE instead of letting them read a dead
        owner's tables."""
        if engine.ingest != "arena":
            raise ValueError("the live server needs an arena-ingest FanoutEngine")
        sc = serving_cfg
        self.eng = engine
        self.ex = engine.ex
        self.layout = engine.arena
        self.fields = self.layout.fields
        # engine buckets (rows each GPU computes per step) and the rows a step
        # takes from THIS rank's arena (scatter fan-out: world x B on rank 0)
        self.buckets: List[int] = sorted(int(b) for b in (buckets or self.ex.buckets))
        self.step_rows: List[int] = [max(1, engine.contrib_rows(B)) for B in self.buckets]
        self.max_request_rows = int(min(sc.max_request_rows, sc.max_queued_rows))
        self.model_name = model_name or sc.model_name
        self.version = sc.version if version is None else version
        self.output_key, self.ids_key, self.wts_key = sc.output_key, sc.ids_key, sc.wts_key
        self.signature_name = sc.signature_name
        depth = int(depth or self.ex.slots)
        # host-side K0 (csrc/runtime/narrow.h): families whose ids all hash with
        # one modulo let the host narrow them to int32 rows while it copies
        # each request (weights stay fp32): 8 instead of 12 bytes per feature
        model = self.ex.model
        m = host_narrow_modulo(model.cfg)
        if narrow is None:  # default: GPU servables (a CPU backend gains nothing from fewer bytes)
            narrow = bool(getattr(sc, "narrow_ingest", True)) and engine.cuda
        self.narrow_modulo = m if narrow else 0
        # ... and models that read only the leading weight columns (one-hot
        # DLRM: the dense features) get only those copied (fewer H2D bytes)
        wc = int(getattr(model, "narrow_weight_cols", lambda: 0)()) if self.narrow_modulo else 0
        self.narrow_wts_cols = wc if 0 < wc < self.fields else 0
        seg = engine.scatter
        n_ar = int(n_arenas or depth + 3)
        if seg is not None and engine.rank == 0:
            # shared-arena scatter: rank 0 batches straight into the segment
            # every rank reads its share from (parallel/shared_scatter.py)
            if seg.n_arenas < max(n_ar, depth + 2):
                raise ValueError(f"shared scatter segment has {seg.n_arenas} arenas, the live server needs {n_ar}")
            self.arenas = [seg.arena(i) for i in range(n_ar)]
        elif engine.cuda:  # pinned, on this rank's NUMA node when it has one (utils/affinity.py)
            from ..utils.affinity import alloc_pinned_arena

            self.arenas = [alloc_pinned_arena(self.layout.capacity) for _ in range(n_ar)]
        else:
            self.arenas = [self.layout.alloc() for _ in range(n_ar)]
        self.config = dict(
            fields=self.fields, ids_key=sc.ids_key, wts_key=sc.wts_key, model_name=self.model_name,
            signature_name=sc.signature_name, output_key=sc.output_key, version=self.version,
            max_batch_rows=min(sc.max_batch_rows * (self.step_rows[-1] // self.buckets[-1] or 1), self.step_rows[-1]),
            batch_timeout_us=sc.batch_timeout_us,
            depth=depth, varint_chunks=self.layout.varint_chunks,
            max_pending=max(64, sc.max_queued_rows // max(1, min(self.buckets))),
            step_timeout_us=int(step_timeout_s * 1e6), peer_timeout_us=int(peer_timeout_s * 1e6),
            start_paused=start_paused, narrow_modulo=self.narrow_modulo, narrow_wts_cols=self.narrow_wts_cols,
            liveness_only=bool(liveness_only and control is not None),
            caller_outputs=["sorted_prediction", "sorted_index"])  # service.RANKED_OUTPUTS
        if engine.cuda:
            from ..ops import hip

            spec = [(R, engine.loop_slots(B)) for B, R in zip(self.buckets, self.step_rows)]
            self.srv = hip().LiveServer(engine.runner(), self.config, spec, self.arenas, control, seg,
                                        self.buckets if seg is not None else None)
            cache = getattr(model, "cache", None)
            if cache is not None and hasattr(cache, "set_step_stream"):
                # the peer-exchange step's kernels all run on the runner's compute
                # stream: replica-cache refreshes run there, stream-ordered with them
                cache.set_step_stream(engine.runner().compute_stream)
        else:
            slots = self.ex.slots
            scores = [[engine.host_out(B, s) for B in self.buckets] for s in range(slots)]
            buckets = self.buckets

            def forward(ai: int, slot: int, b: int) -> None:
                engine.launch(buckets[b], slot, src=self.arenas[ai], nbytes=self.layout.capacity).wait()

            self.srv = native().LiveServer(self.config, self.step_rows, scores, self.arenas, forward, control)
        self.control = control
        self.max_rows = int(self.srv.max_rows)
        self.OVERSIZE = int(native().STATUS_OVERSIZE)
        self.CALLER_PATH = int(native().STATUS_CALLER_PATH)

    # -- fast path: serialized request in, serialized response out -------------
    def predict_raw(self, data: bytes, timeout_s: Optional[float] = None):
        """(code, message, response bytes) straight from the native server."""
        return self.srv.predict(data, float(timeout_s or 0.0))

    def predict_bytes(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        code, msg, resp = self.predict_raw(data, timeout_s)
        if code == 0:
            return resp
        raise ServingError(_code(code), msg)

    # -- slow path: rows -> raw requests of <= one batch -> joined scores ---------
    def _encode(self, ids: torch.Tensor, wts: torch.Tensor) -> bytes:
        return native().encode_predict_request(
            self.model_name, self.signature_name, self.version if self.version >= 0 else None,
            [(self.ids_key, ids.contiguous()), (self.wts_key, wts.contiguous())], True)

    def submit_rows(self, ids: torch.Tensor, wts: torch.Tensor, timeout_s: float = 0.0) -> cf.Future:
        """Future of fp32 scores [rows] for int64 ids / fp32 weights [rows, F]."""
        rows = int(ids.shape[0])
        out: cf.Future = cf.Future()
        if rows == 0:
            out.set_result(torch.empty(0))
            return out
        parts = [(s, min(rows, s + self.max_rows)) for s in range(0, rows, self.max_rows)]
        results: List[Optional[np.ndarray]] = [None] * len(parts)
        state = {"left": len(parts), "failed": False}
        import threading

        lock = threading.Lock()
        from ..wire import schema as pb

        def cb(k, code, msg, resp):
            with lock:
                if state["failed"]:
                    return
                if code != 0:
                    state["failed"] = True
                    out.set_exception(ServingError(_code(code), msg))
                    return
                r = pb.PredictResponse.FromString(resp)
                results[k] = np.asarray(r.outputs[self.output_key].float_val, dtype=np.float32)
                state["left"] -= 1
                if state["left"] == 0:
                    out.set_result(torch.from_numpy(np.concatenate(results)))

        ids = ids.to(torch.int64)
        wts = wts.to(torch.float32)
        for k, (s, e) in enumerate(parts):
            self.srv.submit(self._encode(ids[s:e], wts[s:e]), float(timeout_s or 0.0),
                            lambda code, msg, resp, k=k: cb(k, code, msg, resp))
        return out

    def submit(self, rows: int, fill, deadline_us: int = 0) -> cf.Future:
        """BatchingScheduler-compatible entry: ``fill(ids, wts)`` writes the rows."""
        if rows > self.max_request_rows:
            fut: cf.Future = cf.Future()
            fut.set_exception(ServingError(
                Code.INVALID_ARGUMENT, f"request has {rows} rows; this server accepts at most {self.max_request_rows}"))
            return fut
        ids = torch.empty(rows, self.fields, dtype=torch.int64)
        wts = torch.empty(rows, self.fields, dtype=torch.float32)
        if rows:
            fill(ids, wts)
        timeout_s = max(1e-6, (deadline_us - native().now_us()) * 1e-6) if deadline_us else 0.0
        return self.submit_rows(ids, wts, timeout_s)

    # -- admin -------------------------------------------------------------------
    def run_load(self, requests: Sequence[bytes], **spec) -> dict:
        return self.srv.run_load(list(requests), spec)

    def stats(self) -> dict:
        st = dict(self.srv.stats())
        seg = self.eng.scatter
        if seg is not None:  # shared-arena scatter: what this rank copied for its shares
            st["scatter_h2d_bytes"] = int(seg.h2d_bytes)
            st["scatter_h2d_steps"] = int(seg.h2d_steps)
        cache = getattr(self.eng.ex.model, "cache", None)
        if cache is not None:  # peer exchange: the hot-row replica cache (counted candidates)
            h, m = cache.counts()
            st["hot_cache_rows"] = int(cache.keys.numel())
            st["hot_cache_refreshes"] = int(cache.refreshes)
            st["hot_cache_hits"], st["hot_cache_misses"] = h, m
            st["hot_cache_refresh_failures"] = int(cache.refresh_failures)
            st["hot_cache_refresher_alive"] = int(cache.refresher_alive)
        # the names the monitoring endpoint reads (serving/monitoring.py)
        st.setdefault("batches", st["steps"])
        st.setdefault("batched_rows", st["rows"])
        st.setdefault("rows_served", st["rows"])
        st.setdefault("timeout_batches", st["timeout_steps"])
        st.setdefault("full_batches", st["full_steps"])
        return st

    def resume(self) -> None:
        """Start launching steps (a server built with ``start_paused``)."""
        self.srv.resume()

    @property
    def broken(self) -> bool:
        return bool(self.srv.broken)

    def close(self) -> None:
        self.srv.close()  # every launched step has completed
        release = getattr(self.eng.ex.model, "release", None)
        if release is not None:  # replica-cache refresher + IPC-mapped peer stores
            release()

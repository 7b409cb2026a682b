"""Fault injection for failure-path tests.

The reference has no failure handling at all: mode A rethrows a
CompletionException that kills the requester thread, mode B prints and drops
the request (reference DCNClient.java:158-159, :185-188), and there are no RPC
deadlines (:111-112). This framework has deadlines (batching), shard
fail-over (client/fanout_client.py) and communicator health checks
(serving/cluster.py); these hooks make those paths testable:

    spec = "after:100,kind:error"      # requests 101.. fail with UNAVAILABLE
    spec = "after:0,kind:delay,ms:250" # every request stalls 250 ms
    spec = "after:10,kind:hang"        # requests 11.. never answer (deadline test)

``--inject-fault SPEC`` on the model server wraps its PredictionService;
:class:`FaultyBackend` wraps a client backend.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Optional

from .errors import Code, ServingError


@dataclass
class FaultSpec:
    after: int = 0          # the first `after` requests are served normally
    kind: str = "error"     # error | delay | hang
    ms: float = 0.0         # delay length
    every: int = 1          # inject on every `every`-th request once active

    @classmethod
    def parse(cls, spec: str) -> "FaultSpec":
        f = cls()
        for part in filter(None, (p.strip() for p in spec.split(","))):
            k, _, v = part.partition(":")
            if k == "after":
                f.after = int(v)
            elif k == "kind":
                if v not in ("error", "delay", "hang"):
                    raise ValueError(f"unknown fault kind {v!r}")
                f.kind = v
            elif k == "ms":
                f.ms = float(v)
            elif k == "every":
                f.every = max(1, int(v))
            else:
                raise ValueError(f"unknown fault option {k!r} in {spec!r}")
        return f


class FaultInjector:
    def __init__(self, spec: FaultSpec):
        self.spec = spec
        self.count = 0
        self.injected = 0
        self._lock = threading.Lock()
        self._hang = threading.Event()

    def check(self, timeout_s: Optional[float] = None) -> None:
        """Call once per request; raises / sleeps / blocks per the spec."""
        with self._lock:
            self.count += 1
            n = self.count
        s = self.spec
        if n <= s.after or (n - s.after - 1) % s.every:
            return
        with self._lock:
            self.injected += 1
        if s.kind == "error":
            raise ServingError(Code.UNAVAILABLE, f"injected fault (request {n})")
        if s.kind == "delay":
            time.sleep(s.ms / 1e3)
            return
        # hang: block until the caller's deadline (or forever), then fail
        self._hang.wait(timeout_s)
        raise ServingError(Code.DEADLINE_EXCEEDED, f"injected hang (request {n})")

    def release(self) -> None:
        self._hang.set()


class FaultyService:
    """Wraps a PredictionServiceImpl: Predict goes through the injector."""

    def __init__(self, service, injector: FaultInjector):
        self._svc, self.injector = service, injector

    def predict_bytes(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        self.injector.check(timeout_s)
        return self._svc.predict_bytes(data, timeout_s)

    def predict(self, request, timeout_s: Optional[float] = None):
        self.injector.check(timeout_s)
        return self._svc.predict(request, timeout_s)

    def __getattr__(self, name):
        return getattr(self._svc, name)


class FaultyBackend:
    """Wraps a client Backend (client/backends.py)."""

    def __init__(self, backend, injector: FaultInjector):
        self._be, self.injector = backend, injector
        self.name = f"faulty({backend.name})"

    def predict(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        self.injector.check(timeout_s)
        return self._be.predict(data, timeout_s)

    def close(self) -> None:
        self.injector.release()
        self._be.close()

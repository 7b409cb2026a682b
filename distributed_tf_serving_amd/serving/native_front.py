"""Native gRPC front door: ``tensorflow.serving.PredictionService`` served by
C++ event loops (csrc/net/h2_server.cpp: HTTP/2 framing, HPACK, flow control,
gRPC messages, deadlines, status trailers) with Predict handed straight to the
servable's native live server.

The grpcio front door (serving/grpc_server.py) runs every RPC through Python
under the GIL - about 170-200 us of serialized work per call, a 5-6 k RPC/s
ceiling (profiles/grpc_ceiling.md). Here a Predict never touches Python: the
event-loop thread that decoded it calls ``LiveServer::submit`` (validation,
admission into the dynamic batch, one copy into the pinned arena), and the
live server's completer hands the encoded PredictResponse back to the loop.
The other four RPCs - and Predicts the fast path returns to its caller
(ranked outputs, requests larger than one batch) - go to
:func:`make_fallback`, which calls the same :class:`PredictionServiceImpl` as
the grpcio door, on a few worker threads.

Reference counterpart: the TF-Serving gRPC endpoint that the reference client
calls, ``stub.predict`` over plaintext HTTP/2 (reference DCNClient.java:111-112,
:118-125; pom.xml:83-92). Unmodified gRPC clients (grpcio, the reference's
gRPC-java) interoperate: they speak h2c with prior knowledge on insecure
channels.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Optional, Tuple

from ..wire import schema as pb
from .errors import ServingError

log = logging.getLogger(__name__)


def make_fallback(service):
    """(path, request bytes, timeout_s) -> (grpc status, message, response
    bytes) over ``service`` - the slow-path handler the native loops call."""
    M = pb.METHODS
    prefix = "/" + pb.SERVICE_NAME + "/"

    def handle(path: str, data: bytes, timeout_s: float) -> Tuple[int, str, bytes]:
        t = timeout_s if timeout_s and timeout_s > 0 else None
        if not path.startswith(prefix) or path[len(prefix):] not in M:
            return 12, f"unknown method {path}", b""
        name = path[len(prefix):]
        try:
            if name == "Predict":
                return 0, "", service.predict_bytes(data, t)
            req = M[name][0].FromString(data)
            if name == "Classify":
                resp = service.classify(req, t)
            elif name == "Regress":
                resp = service.regress(req, t)
            elif name == "MultiInference":
                resp = service.multi_inference(req, t)
            else:
                resp = service.get_model_metadata(req)
            return 0, "", resp.SerializeToString()
        except ServingError as e:
            return int(e.code), e.message, b""
        except Exception as e:  # noqa: BLE001 - any other failure is INTERNAL, never a dead loop
            log.exception("RPC %s failed", path)
            return 13, str(e), b""

    return handle


class NativeGrpcFront:
    """Same surface as :class:`serving.grpc_server.GrpcFrontDoor`
    (``port`` / ``start`` / ``stop`` / ``wait``)."""

    def __init__(self, service, live, port: int = 9999, host: str = "0.0.0.0", threads: int = 4,
                 fallback_threads: int = 4, max_message_mb: int = 64):
        """``live``: the servable's :class:`serving.live.LiveScheduler`;
        ``service`` None serves Predict's fast path only (UNIMPLEMENTED for
        the rest, INTERNAL for what the fast path hands back)."""
        self.service = service
        self.live = live
        mod = type(live.srv).__module__
        from ..ops import hip, native

        m = hip() if mod.endswith("_hip") else native()
        fb = make_fallback(service) if service is not None else None  # None: Predict fast path only
        self._front = m.GrpcFront(live.srv, int(port), host, int(threads), fb, int(fallback_threads),
                                  int(max_message_mb) << 20)
        self.port = int(self._front.port)
        self._done = threading.Event()

    def start(self) -> "NativeGrpcFront":
        log.info("PredictionService (native h2c) listening on port %d", self.port)
        return self

    def stats(self) -> dict:
        return dict(self._front.stats())

    def stop(self, grace: Optional[float] = None) -> None:
        self._front.stop()
        self._done.set()

    def wait(self) -> None:
        while not self._done.wait(1.0):
            pass

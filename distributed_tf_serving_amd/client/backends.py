"""Transports a client can fan out over.

A backend takes a serialized PredictRequest and returns a serialized
PredictResponse, synchronously (``predict``) - the client's dispatcher pool
provides the asynchrony, like the reference's blocking stubs on a
CompletableFuture pool (reference DCNClient.java:111-112, :148-156).

``InProcessBackend``  calls a PredictionServiceImpl in the same process.
``GrpcBackend``       plaintext gRPC channel to a PredictionService
                      (ours or TF-Serving), one channel per host, created once
                      (reference getChannels, DCNClient.java:118-125) and shut
                      down explicitly (the reference only awaits, :127-135).
"""
from __future__ import annotations

from typing import Optional

from ..wire import schema as pb

PREDICT_PATH = f"/{pb.SERVICE_NAME}/Predict"


class Backend:
    name = "backend"

    def predict(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:  # pragma: no cover
        raise NotImplementedError

    def close(self) -> None:
        pass


class InProcessBackend(Backend):
    def __init__(self, service, name: str = "inproc"):
        self.service, self.name = service, name

    def predict(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        return self.service.predict_bytes(data, timeout_s)


class GrpcBackend(Backend):
    def __init__(self, target: str, max_message_mb: int = 64):
        import grpc

        self.name = target
        opts = [("grpc.max_receive_message_length", max_message_mb << 20),
                ("grpc.max_send_message_length", max_message_mb << 20)]
        self.channel = grpc.insecure_channel(target, options=opts)
        self._call = self.channel.unary_unary(PREDICT_PATH, request_serializer=None, response_deserializer=None)
        self._meta = {}

    def predict(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        return self._call(data, timeout=timeout_s)

    def call(self, method: str, request, timeout_s: Optional[float] = None):
        """Any PredictionService RPC with message objects (Classify, Regress, ...)."""
        req_cls, resp_cls = pb.METHODS[method]
        fn = self._meta.get(method)
        if fn is None:
            fn = self._meta[method] = self.channel.unary_unary(
                f"/{pb.SERVICE_NAME}/{method}", request_serializer=req_cls.SerializeToString,
                response_deserializer=resp_cls.FromString)
        return fn(request, timeout=timeout_s)

    def close(self) -> None:
        self.channel.close()

"""gRPC front door: ``tensorflow.serving.PredictionService`` on a TCP port.

There is no grpc codegen in this image (no grpc_tools), so the service is
registered with ``grpc.method_handlers_generic_handler`` under the exact method
paths TF-Serving uses (``/tensorflow.serving.PredictionService/Predict``...).
An unmodified TF-Serving client - including the reference Java DCNClient
(reference DCNClient.java:111-112, plaintext, port 9999) - can talk to it.

Predict takes the serialized request bytes straight into the native codec
(no python protobuf parse on the hot path); the other RPCs use message objects.
This front door is for compatibility: inside a node the fan-out between GPUs
is RCCL over xGMI (parallel/fanout.py), never gRPC.
"""
from __future__ import annotations

import concurrent.futures as cf
import logging
import time
from typing import Optional

import grpc

from ..wire import schema as pb
from .errors import ServingError
from .service import PredictionServiceImpl

log = logging.getLogger(__name__)

_ident = lambda b: b  # noqa: E731 - raw bytes in / out


def _wrap(fn, api: str = "", metrics=None, ctx_timeout=True):
    def handler(request, context):
        t0 = time.perf_counter()
        status = "OK"
        try:
            t = context.time_remaining() if ctx_timeout else None
            return fn(request, t if t is not None and t < 1e8 else None)
        except ServingError as e:
            status = e.grpc_code().name
            context.abort(e.grpc_code(), e.message)
        except Exception as e:  # noqa: BLE001
            status = "INTERNAL"
            log.exception("RPC failed")
            context.abort(grpc.StatusCode.INTERNAL, str(e))
        finally:
            if metrics is not None:
                metrics.observe(api, status, t0)

    return handler


def make_handler(service: PredictionServiceImpl, metrics=None) -> grpc.GenericRpcHandler:
    M = pb.METHODS

    def msg_handler(name, fn):
        req_cls, resp_cls = M[name]
        return grpc.unary_unary_rpc_method_handler(
            _wrap(fn, name, metrics), request_deserializer=req_cls.FromString,
            response_serializer=resp_cls.SerializeToString)

    handlers = {
        "Predict": grpc.unary_unary_rpc_method_handler(
            _wrap(lambda data, t: service.predict_bytes(data, t), "Predict", metrics), request_deserializer=_ident,
            response_serializer=_ident),
        "Classify": msg_handler("Classify", lambda r, t: service.classify(r, t)),
        "Regress": msg_handler("Regress", lambda r, t: service.regress(r, t)),
        "MultiInference": msg_handler("MultiInference", lambda r, t: service.multi_inference(r, t)),
        "GetModelMetadata": msg_handler("GetModelMetadata", lambda r, t: service.get_model_metadata(r)),
    }
    return grpc.method_handlers_generic_handler(pb.SERVICE_NAME, handlers)


class GrpcFrontDoor:
    def __init__(self, service: PredictionServiceImpl, port: int = 9999, host: str = "0.0.0.0",
                 max_workers: int = 32, max_message_mb: int = 64, metrics=None):
        self.service = service
        self.metrics = metrics  # serving/monitoring.py ServingMetrics (optional)
        opts = [("grpc.max_receive_message_length", max_message_mb << 20),
                ("grpc.max_send_message_length", max_message_mb << 20)]
        self.server = grpc.server(cf.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="dtfs-grpc"),
                                  options=opts)
        self.server.add_generic_rpc_handlers((make_handler(service, metrics),))
        self.port = self.server.add_insecure_port(f"{host}:{port}")
        if self.port == 0:
            raise RuntimeError(f"could not bind {host}:{port}")

    def start(self) -> "GrpcFrontDoor":
        self.server.start()
        log.info("PredictionService listening on port %d", self.port)
        return self

    def stop(self, grace: Optional[float] = 1.0) -> None:
        self.server.stop(grace).wait()

    def wait(self) -> None:
        self.server.wait_for_termination()

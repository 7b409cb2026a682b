"""Multi-GPU model server: one front door fanning candidates out to every GPU.

The reference client fans each request's candidates out to N TF-Serving hosts
itself (reference DCNClient.java:46-74 split, :146-164 dispatch + join). Here
that fan-out moves inside one node: rank 0 runs the PredictionService front
door (gRPC and/or in-process) and the dynamic batcher; every batch of world x B
candidate rows is scattered over the GPUs by RCCL (parallel/fanout.py, scatter
mode), each GPU scores its B rows, and the scores are gathered back. Ranks > 0
run :func:`ClusterServer.serve_follower`: per step they receive the step's
(bucket, slot) over a small gloo control channel and join its collectives.

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 -m distributed_tf_serving_amd.serving.cluster \\
        --preset deepfm_fanout4 --port 9999

Failure handling: the control channel has a timeout (a dead rank 0 ends the
followers); the native RCCL communicators are polled for asynchronous errors
(:meth:`ClusterServer.health`) and aborted on shutdown.
"""
from __future__ import annotations

import argparse
import collections
import datetime
import logging
import signal
from typing import Optional

import torch
import torch.distributed as dist

from ..config import Config, load_preset
from ..parallel.dist import DistContext, init_from_env, shutdown
from ..utils.gc_tuning import tune_for_serving
from .registry import ModelRegistry
from .server import build_engine, build_servable
from .service import PredictionServiceImpl

log = logging.getLogger(__name__)

STOP = -1


class StepControl:
    """Rank 0 -> followers: (bucket, slot) of every step, over a CPU gloo group
    (a 16-byte broadcast per step; the data itself moves over RCCL)."""

    def __init__(self, ctx: DistContext, timeout_s: float = 3600.0):
        self.ctx = ctx
        self.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
        self._buf = torch.zeros(2, dtype=torch.int64)

    def send(self, B: int, slot: int) -> None:
        self._buf[0], self._buf[1] = int(B), int(slot)
        dist.broadcast(self._buf, src=0, group=self.group)

    def recv(self):
        dist.broadcast(self._buf, src=0, group=self.group)
        return int(self._buf[0]), int(self._buf[1])

    def stop(self) -> None:
        self.send(STOP, 0)


class ClusterServer:
    """Every rank constructs one (collective); rank 0 serves, the rest follow."""

    def __init__(self, cfg: Config, ctx: DistContext, slots: int = 3, self_check: bool = True):
        self.cfg, self.ctx = cfg, ctx
        self.rank = ctx.rank if ctx.is_distributed else 0
        mode = "scatter" if ctx.is_distributed else "local"
        self.engine = build_engine(cfg, ctx.device, slots, ctx=ctx, mode=mode)
        if self_check and mode != "local":
            B = self.engine.ex.buckets[-1]
            if not self.engine.self_check(B):
                log.warning("fan-out self-check failed on some rank; serving on the torch.distributed path")
        self.ctrl = StepControl(ctx) if ctx.is_distributed else None
        self.depth = max(1, slots - 1)
        self.registry: Optional[ModelRegistry] = None
        self.service: Optional[PredictionServiceImpl] = None
        self.front = None
        self.metrics = None
        self.steps_followed = 0
        if self.rank == 0:
            on_launch = self.ctrl.send if self.ctrl is not None else None
            self.registry = ModelRegistry()
            self.registry.load(build_servable(cfg, slots=slots, engine=self.engine, on_launch=on_launch))
            self.service = PredictionServiceImpl(self.registry, cfg.serving.request_timeout_s)

    # -- rank 0 -------------------------------------------------------------------
    def start_grpc(self, port: int = 9999, host: str = "0.0.0.0", max_workers: int = 32,
                   monitoring_port: Optional[int] = None) -> int:
        """monitoring_port: also serve Prometheus metrics (serving/monitoring.py)."""
        from .grpc_server import GrpcFrontDoor
        from .monitoring import ServingMetrics

        assert self.rank == 0, "only rank 0 is a front door"
        self.metrics = ServingMetrics(self.registry)
        self.front = GrpcFrontDoor(self.service, port=port, host=host, max_workers=max_workers,
                                   metrics=self.metrics).start()
        if monitoring_port is not None:
            self.metrics.serve_http(monitoring_port, host)
        return self.front.port

    # -- ranks > 0 ----------------------------------------------------------------
    def serve_follower(self) -> int:
        """Join every step rank 0 launches until it sends STOP; returns steps served."""
        assert self.rank != 0 and self.ctrl is not None
        inflight = collections.deque()
        while True:
            B, slot = self.ctrl.recv()
            if B == STOP:
                break
            inflight.append(self.engine.launch(B, slot, nbytes=0 if self.engine.ingest == "arena" else None))
            if len(inflight) >= self.depth:
                inflight.popleft().wait()
                self.steps_followed += 1
        while inflight:
            inflight.popleft().wait()
            self.steps_followed += 1
        return self.steps_followed

    def health(self) -> Optional[str]:
        """First asynchronous communicator error of this rank (None = healthy)."""
        return self.engine.comm_error() if self.engine.native_fanout_active else None

    def stop(self) -> None:
        if self.rank == 0:
            if self.metrics is not None:
                self.metrics.stop()
            if self.front is not None:
                self.front.stop()
                self.front = None
            if self.registry is not None:
                self.registry.close()  # drains the batcher: every launched step completes
            if self.ctrl is not None:
                self.ctrl.stop()


def main(argv=None):
    ap = argparse.ArgumentParser(description="multi-GPU CTR model server (rank 0 = PredictionService front door)")
    ap.add_argument("--preset", default="deepfm_fanout4")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--grpc-workers", type=int, default=32)
    ap.add_argument("--monitoring-port", type=int, default=None,
                    help="serve Prometheus metrics over HTTP on this port (rank 0)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    ctx = init_from_env()
    srv = ClusterServer(load_preset(a.preset), ctx)
    try:
        if srv.rank == 0:
            port = srv.start_grpc(a.port, a.host, a.grpc_workers, a.monitoring_port)
        tune_for_serving()  # every rank: a GC pause on a follower stalls the step's collectives too
        if srv.rank == 0:
            print(f"serving on port {port} over {ctx.world} GPU(s)", flush=True)
            signal.signal(signal.SIGTERM, lambda *_: srv.front.stop() if srv.front else None)
            try:
                srv.front.wait()
            except KeyboardInterrupt:
                pass
        else:
            srv.serve_follower()
    finally:
        srv.stop()
        shutdown()


if __name__ == "__main__":
    main()

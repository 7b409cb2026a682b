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

Failure handling (the reference has none: a failed shard kills the requester
thread, reference DCNClient.java:158-159, :185-188):

* every GPU step wait is bounded (``FanoutEngine.step_timeout_s``) and polls
  the RCCL communicators' asynchronous errors; a step that does not finish
  marks rank 0's scheduler BROKEN: in-flight and queued requests fail
  UNAVAILABLE, later ones immediately, the communicators are aborted and the
  followers are told to stop (best effort);
* a launch that fails after the followers were told about the step also
  breaks the cluster (the ranks' collective sequences no longer match);
* rank 0 sends a heartbeat on the control channel when idle; a follower that
  hears nothing for ``control_timeout_s`` (rank 0 is gone) exits non-zero;
  a follower that loses its peers fails its step wait and exits non-zero;
* a watchdog thread on rank 0 polls :meth:`ClusterServer.health`.
"""
from __future__ import annotations

import argparse
import collections
import datetime
import logging
import os
import signal
import threading
import time
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
HEARTBEAT = 0  # bucket 0: no step, rank 0 is alive


class StepControl:
    """Rank 0 -> followers: (bucket, slot) of every step, over a CPU gloo group
    (a 16-byte broadcast per step; the data itself moves over RCCL). Rank 0
    sends heartbeats while idle, so a follower can tell an idle server from a
    dead one within ``timeout_s``."""

    def __init__(self, ctx: DistContext, timeout_s: float = 30.0, heartbeat_s: float = 1.0):
        self.ctx = ctx
        self.timeout_s = timeout_s
        self.heartbeat_s = heartbeat_s
        self.group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=timeout_s))
        self._buf = torch.zeros(2, dtype=torch.int64)
        self._lock = threading.Lock()
        self._last_send = time.monotonic()
        self._hb: Optional[threading.Thread] = None
        self._stop = threading.Event()

    def send(self, B: int, slot: int) -> None:
        with self._lock:
            self._buf[0], self._buf[1] = int(B), int(slot)
            dist.broadcast(self._buf, src=0, group=self.group)
            self._last_send = time.monotonic()

    def recv(self):
        dist.broadcast(self._buf, src=0, group=self.group)
        return int(self._buf[0]), int(self._buf[1])

    def start_heartbeat(self) -> None:
        def run():
            while not self._stop.wait(self.heartbeat_s / 2):
                if time.monotonic() - self._last_send >= self.heartbeat_s:
                    try:
                        self.send(HEARTBEAT, 0)
                    except Exception as e:  # noqa: BLE001 - a follower is gone
                        log.error("control heartbeat failed: %s", e)
                        return

        self._hb = threading.Thread(target=run, name="dtfs-heartbeat", daemon=True)
        self._hb.start()

    def stop(self) -> None:
        self._stop.set()
        if self._hb is not None:
            self._hb.join(timeout=5)
        self.send(STOP, 0)


class ClusterServer:
    """Every rank constructs one (collective); rank 0 serves, the rest follow."""

    def __init__(self, cfg: Config, ctx: DistContext, slots: int = 3, self_check: bool = True,
                 control_timeout_s: float = 30.0, step_timeout_s: Optional[float] = None,
                 follower_fault: Optional[dict] = None):
        self.cfg, self.ctx = cfg, ctx
        self.rank = ctx.rank if ctx.is_distributed else 0
        mode = "scatter" if ctx.is_distributed else "local"
        self.engine = build_engine(cfg, ctx.device, slots, ctx=ctx, mode=mode)
        if step_timeout_s is not None:
            self.engine.step_timeout_s = step_timeout_s
        if self_check and mode != "local":
            B = self.engine.ex.buckets[-1]
            if not self.engine.self_check(B):
                log.warning("fan-out self-check failed on some rank; serving on the torch.distributed path")
        self.ctrl = StepControl(ctx, timeout_s=control_timeout_s) if ctx.is_distributed else None
        self.depth = max(1, slots - 1)
        self.registry: Optional[ModelRegistry] = None
        self.service: Optional[PredictionServiceImpl] = None
        self.front = None
        self.metrics = None
        self.steps_followed = 0
        self.follower_fault = follower_fault or {}
        self._watchdog: Optional[threading.Thread] = None
        self._stopping = threading.Event()
        self.sched = None
        if self.rank == 0:
            on_launch = self.ctrl.send if self.ctrl is not None else None
            self.registry = ModelRegistry()
            servable = build_servable(cfg, slots=slots, engine=self.engine, on_launch=on_launch)
            self.sched = servable.scheduler
            if hasattr(self.sched, "on_broken"):
                self.sched.on_broken = self._on_broken
            self.registry.load(servable)
            self.service = PredictionServiceImpl(self.registry, cfg.serving.request_timeout_s)
            if self.ctrl is not None:
                self.ctrl.start_heartbeat()
                self._watchdog = threading.Thread(target=self._watch, name="dtfs-watchdog", daemon=True)
                self._watchdog.start()

    # -- failure handling (rank 0) ----------------------------------------------
    def _on_broken(self, reason: str) -> None:
        log.error("cluster broken: %s - aborting communicators, stopping followers", reason)
        try:
            self.engine.abort()
        except Exception:  # noqa: BLE001
            log.exception("communicator abort failed")

    def _watch(self, period_s: float = 0.5) -> None:
        while not self._stopping.wait(period_s):
            err = self.health()
            if err and self.sched is not None and hasattr(self.sched, "mark_broken"):
                self.sched.mark_broken(f"communicator error: {err}")
                return

    @property
    def broken(self) -> Optional[str]:
        return getattr(self.sched, "broken", None)

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
        """Join every step rank 0 launches until it sends STOP; returns steps
        served. Raises when rank 0 goes silent or a step cannot finish."""
        assert self.rank != 0 and self.ctrl is not None
        inflight = collections.deque()
        fault_after = int(self.follower_fault.get("after", -1))
        launched = 0
        while True:
            B, slot = self.ctrl.recv()  # times out (raises) if rank 0 is gone
            if B == STOP:
                break
            if B == HEARTBEAT:
                continue
            if fault_after >= 0 and launched >= fault_after:
                log.error("fault injection: follower rank %d exits before step %d", self.rank, launched)
                os._exit(int(self.follower_fault.get("code", 17)))
            inflight.append(self.engine.launch(B, slot, nbytes=0 if self.engine.ingest == "arena" else None))
            launched += 1
            if len(inflight) >= self.depth:
                inflight.popleft().wait()  # bounded (engine.step_timeout_s)
                self.steps_followed += 1
        while inflight:
            inflight.popleft().wait()
            self.steps_followed += 1
        return self.steps_followed

    def health(self) -> Optional[str]:
        """First asynchronous communicator error of this rank (None = healthy)."""
        return self.engine.comm_error() if self.engine.native_fanout_active else None

    def stop(self) -> None:
        self._stopping.set()
        if self.rank == 0:
            if self.metrics is not None:
                self.metrics.stop()
            if self.front is not None:
                self.front.stop()
                self.front = None
            if self.registry is not None:
                self.registry.close()  # drains the batcher: every launched step completes
            if self.ctrl is not None and not self.broken:
                try:
                    self.ctrl.stop()
                except Exception as e:  # noqa: BLE001 - followers already gone
                    log.warning("could not stop the followers: %s", e)


def main(argv=None):
    ap = argparse.ArgumentParser(description="multi-GPU CTR model server (rank 0 = PredictionService front door)")
    ap.add_argument("--preset", default="deepfm_fanout4")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--grpc-workers", type=int, default=32)
    ap.add_argument("--monitoring-port", type=int, default=None,
                    help="serve Prometheus metrics over HTTP on this port (rank 0)")
    ap.add_argument("--control-timeout-s", type=float, default=30.0,
                    help="a follower that hears nothing from rank 0 this long exits")
    ap.add_argument("--step-timeout-s", type=float, default=30.0,
                    help="a GPU step not finished this long breaks the cluster (UNAVAILABLE)")
    ap.add_argument("--no-gc-freeze", action="store_true",
                    help="leave CPython's cyclic GC at its defaults (utils/gc_tuning.py)")
    ap.add_argument("--peer-comm", type=int, default=None,
                    help="one-shot peer exchange for fan-out messages of at most this many bytes per peer "
                         "(1 = 64 KiB, 0 = RCCL only; default: $DTFS_PEER_COMM or 0)")
    a = ap.parse_args(argv)
    if a.peer_comm is not None:
        os.environ["DTFS_PEER_COMM"] = str(max(0, a.peer_comm))
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    ctx = init_from_env(timeout_s=max(60.0, a.control_timeout_s))
    srv = ClusterServer(load_preset(a.preset), ctx, control_timeout_s=a.control_timeout_s,
                        step_timeout_s=a.step_timeout_s)
    rc = 0
    try:
        if not a.no_gc_freeze:  # every rank, after warm-up, before traffic: a GC pause on a
            tune_for_serving()  # follower stalls the step's collectives too
        if srv.rank == 0:
            port = srv.start_grpc(a.port, a.host, a.grpc_workers, a.monitoring_port)
            print(f"serving on port {port} over {ctx.world} GPU(s)", flush=True)
            signal.signal(signal.SIGTERM, lambda *_: srv.front.stop() if srv.front else None)
            try:
                srv.front.wait()
            except KeyboardInterrupt:
                pass
        else:
            srv.serve_follower()
    except Exception:  # noqa: BLE001 - a follower that lost rank 0 / its peers
        log.exception("rank %d failed", srv.rank)
        rc = 3
    finally:
        srv.stop()
        if rc == 0:
            shutdown()
    return rc


if __name__ == "__main__":
    raise SystemExit(main())

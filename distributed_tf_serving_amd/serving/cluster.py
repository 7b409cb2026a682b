"""Multi-GPU model server: requests fanned out over every GPU of the node.

The reference client fans each request's candidates out to N TF-Serving hosts
itself (reference DCNClient.java:46-74 split, :146-164 dispatch + join). Here
that fan-out moves inside one node, onto the native live server of every rank
(csrc/runtime/live_server.cpp):

``scatter``   rank 0 runs the PredictionService front door (gRPC and/or
              in-process); each batch of up to world x B candidate rows is
              split evenly over the GPUs. By default (``serving.scatter_path:
              shared``) rank 0 batches into shared request arenas every rank
              maps: each GPU DMAs only its share over its own PCIe link and
              writes its scores into rank 0's shared output, no collective
              (csrc/runtime/shared_scatter.h); ``rccl`` scatters packed rows
              (RCCL / the one-shot peer kernel) and gathers the scores back.
``alltoall``  every rank is a front door (gRPC port + rank); each rank's rows
              are split over all GPUs and the scores return to it.
``local``     every rank is a front door and scores its own requests on its
              own GPU. With a sharded-table model (DLRM, BASELINE config 4) the
              tables live sharded over the ranks and each rank's steps read the
              other ranks' shards where they live (the peer exchange:
              IPC-mapped stores, parallel/embedding_sharding.py): no collective
              in the step, but every rank depends on every table owner. The
              step control then carries liveness only (heartbeats + the broken
              flag, no step agreement): a dead owner turns every rank's requests
              into UNAVAILABLE within ``control_timeout_s``, and ``--recover``
              re-plans the tables over the survivors (their rows are rebuilt
              from the tables' hashed initialisation, so scores do not change).

Steps are agreed through a shared-memory step control (parallel/control.py,
csrc/runtime/step_control.h): a step runs only when some rank has requests
(an idle cluster launches nothing), at the smallest padding bucket that holds
every rank's batch, so a lone request costs a small step, not a full one.
No Python runs per step or per request on any rank.

    python -m distributed_tf_serving_amd.serving.launch --nproc-per-node 4 -- \\
        -m distributed_tf_serving_amd.serving.cluster --preset deepfm_fanout4 --port 9999

Front doors are the C++ h2c gRPC server by default (``--front native``,
serving/native_front.py: Predict straight into the live server) or grpcio.

Failure handling (the reference has none: a failed shard kills the requester
thread, reference DCNClient.java:158-159, :185-188):

* every GPU step wait is bounded and polls the communicators' asynchronous
  errors; a rank whose step does not finish, or that cannot agree a step with
  its peers within the step timeout, breaks the cluster (a sticky flag in the
  shared segment): in-flight and queued requests fail UNAVAILABLE, later ones
  immediately, and the communicators are aborted so no peer hangs;
* every rank's watcher thread heartbeats into the segment; a rank silent for
  ``peer_timeout_s`` (a dead process) breaks the cluster the same way;
* with ``recover=True`` the survivors then rebuild the cluster among
  themselves (fresh step control and communicators, candidates re-split over
  the survivors, same processes) and resume serving: the requests in flight
  when the rank died fail UNAVAILABLE once, later ones succeed (SURVEY.md
  §5.3). No rank leads the rebuild: every survivor proposes the next epoch's
  members through the job's key-value store and the first proposal wins
  (``compare_set``), so any rank may die - rank 0 included - as long as the
  store outlives it. ``serving/launch.py`` hosts the store in the launcher
  process (torchrun's static rendezvous also keeps it in its agent, but the
  agent tears every rank down once one fails). In ``scatter`` mode rank 0 is
  the only front door: its death leaves nothing to serve, the followers exit.
"""
from __future__ import annotations

import argparse
import datetime
import logging
import os
import signal
import threading
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from ..config import Config, load_preset
from ..parallel.control import create_control, default_store
from ..parallel.dist import DistContext, init_from_env, shutdown
from ..utils.gc_tuning import tune_for_serving
from .registry import ModelRegistry
from .server import build_engine, build_servable
from .service import PredictionServiceImpl

log = logging.getLogger(__name__)


class ClusterServer:
    """Every rank constructs one (collective at start-up); the front-door
    rank(s) serve, the others follow until ``stop``."""

    def __init__(self, cfg: Config, ctx: DistContext, slots: int = 3, self_check: bool = True,
                 control_timeout_s: float = 30.0, step_timeout_s: Optional[float] = None,
                 follower_fault: Optional[dict] = None, mode: str = "scatter", recover: bool = False):
        self.cfg, self.ctx = cfg, ctx
        self.rank = ctx.rank if ctx.is_distributed else 0
        self.world = ctx.world if ctx.is_distributed else 1
        self.orig_rank = self.rank  # rank in the original job (the current epoch's rank is self.rank)
        self._store = default_store() if self.world > 1 else None
        self.mode = mode if self.world > 1 else "local"
        if self.mode not in ("scatter", "alltoall", "local"):
            raise ValueError("mode must be scatter, alltoall or local")
        if step_timeout_s is not None:
            cfg.serving.step_timeout_s = float(step_timeout_s)
        cfg.serving.peer_timeout_s = float(control_timeout_s)
        self.slots = slots
        self.self_check_on = self_check
        self.follower_fault = follower_fault or {}
        self.recover_on = recover
        self.epoch = 0
        self.members: List[int] = list(range(self.world))  # original ranks serving in this epoch
        self.registry: Optional[ModelRegistry] = None
        self.service: Optional[PredictionServiceImpl] = None
        self.front = None
        self.metrics = None
        self._stopping = threading.Event()
        self._lock = threading.RLock()
        self.recoveries = 0
        self._injected_comm_error: Optional[str] = None
        self.engine = self.ctl = self.sched = None
        self._build(ctx, first=True, store=self._store)
        if self.serves and self.world > 1:
            self._watchdog = threading.Thread(target=self._watch, name="dtfs-watchdog", daemon=True)
            self._watchdog.start()

    # -- construction -------------------------------------------------------------
    @property
    def serves(self) -> bool:
        """This rank is a front door (rank 0; every rank in alltoall / local mode)."""
        return self.rank == 0 or self.mode in ("alltoall", "local")

    def _module(self):
        from ..ops import hip, native

        return hip() if self.ctx.device.type == "cuda" else native()

    def _build(self, ctx: DistContext, first: bool, store=None, model=None) -> None:
        """Engine + step control + live server of this rank for ``ctx`` (the
        original job, or the survivors after a rebuild)."""
        world = ctx.world if ctx.is_distributed else 1
        mode = self.mode if world > 1 else "local"
        group = None
        if world > 1 and ctx.device.type != "cuda":
            # the step's gloo collectives run on the live server's launcher
            # thread: their own group, never interleaved with other traffic
            group = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=self.cfg.serving.step_timeout_s))
        eng = build_engine(self.cfg, ctx.device, self.slots, ctx=ctx, mode=mode, group=group, model=model,
                           scatter_tag=f"cluster/{self.epoch}", store=store)
        eng.step_timeout_s = self.cfg.serving.step_timeout_s
        if self.self_check_on and mode != "local":
            B = eng.ex.buckets[-1]
            if not eng.self_check(B, seed=self.epoch):
                raise RuntimeError("fan-out self-check failed: the native step's scores differ from a local forward")
        ctl = None
        # lockstep engines agree every step; independent ranks (local mode:
        # the peer exchange's table owners) share the segment for liveness only
        liveness_only = world > 1 and not eng.lockstep and mode == "local"
        if world > 1 and (eng.lockstep or liveness_only):
            ctl = create_control(self._module(), world, ctx.rank, store=store,
                                 prefix=f"dtfs/ctl/cluster/{self.epoch}")
        servable = build_servable(self.cfg, slots=self.slots, engine=eng, control=ctl, liveness_only=liveness_only)
        with self._lock:
            self.engine, self.ctl, self.sched, self.ctx = eng, ctl, servable.scheduler, ctx
            self.rank, self.world = (ctx.rank, world) if world > 1 else (0, 1)
            if self.serves:
                if self.registry is None:
                    self.registry = ModelRegistry()
                    self.registry.load(servable)
                    self.service = PredictionServiceImpl(self.registry, self.cfg.serving.request_timeout_s)
                else:
                    self.registry.replace(servable)
        if ctl is not None:
            if world > 1 and dist.is_initialized():
                dist.barrier(group=group)  # every rank finished its start-up collectives
            servable.scheduler.resume()

    # -- failure handling -----------------------------------------------------------
    def _watch(self, period_s: float = 0.05) -> None:
        """Front door: turn an asynchronous communicator error into a broken
        cluster, and (``recover``) rebuild over the survivors."""
        while not self._stopping.wait(period_s):
            err = self.health()
            if err and self.ctl is not None and self.ctl.broken_by < 0:
                log.error("communicator error on rank %d: %s", self.rank, err)
                self.ctl.mark_broken(self.rank)  # the live server's watcher breaks it (even when idle)
            if self.broken and self.recover_on and not self._stopping.is_set():
                try:
                    if not self._recover():
                        return
                except Exception:  # noqa: BLE001
                    log.exception("cluster recovery failed; staying unavailable")
                    return

    @property
    def broken(self) -> Optional[str]:
        s = self.sched
        if s is None or not getattr(s, "broken", False):
            return None
        return s.stats().get("error") or "broken"

    def health(self) -> Optional[str]:
        """First asynchronous communicator error of this rank (None = healthy)."""
        if self._injected_comm_error:
            return self._injected_comm_error
        return self.engine.comm_error() if self.engine is not None and self.engine.native_fanout_active else None

    def inject_comm_error(self, msg: str = "injected communicator error") -> None:
        """Fault injection (serving/faults.py family): report ``msg`` as this
        rank's asynchronous communicator error until the next rebuild."""
        self._injected_comm_error = msg

    # -- recovery (serving/cluster.py docstring) ----------------------
    def _survivors(self) -> List[int]:
        """Current-epoch ranks whose heartbeat is fresh. A dead process stops
        beating; a live one beats every few ms even while its step is stuck."""
        ctl, lim = self.ctl, self.cfg.serving.peer_timeout_s
        return [r for r in range(ctl.world) if r == ctl.rank or ctl.heartbeat_age(r) < lim]

    def _recover(self) -> bool:
        """Any rank of a broken cluster: agree on the next epoch's members and
        rebuild if this rank is one of them (False: it was left out, or the
        scatter front door is gone).

        Every survivor proposes the ranks whose heartbeat is fresh; the first
        proposal to reach the store is the epoch's membership (``compare_set``
        on a fresh key), so survivors with different views still agree and no
        leader has to be alive. A rank that breaks before the dead peer's
        heartbeat is stale (a stuck step) waits up to ``peer_timeout_s`` for
        it, unless a proposal is already there."""
        e = self.epoch + 1
        key = f"dtfs/recover/{e}"
        if not self._store.check([key]):
            deadline = time.monotonic() + self.cfg.serving.peer_timeout_s
            alive = self._survivors()
            while len(alive) == self.ctl.world and time.monotonic() < deadline and not self._store.check([key]):
                time.sleep(0.05)
                alive = self._survivors()
            self._store.compare_set(key, "", ",".join(str(self.members[r]) for r in alive))
        members = [int(x) for x in self._store.get(key).decode().split(",")]
        self.ctl.bump_epoch()  # ranks blocked on the old segment wake up and look for the proposal
        if self.orig_rank not in members:
            log.error("rank %d was left out of epoch %d", self.orig_rank, e)
            return False
        if self.mode == "scatter" and self.members[0] not in members:
            log.error("the scatter front door (rank %d) is gone: nothing left to serve", self.members[0])
            return False
        log.warning("rebuilding the cluster over ranks %s (epoch %d)", members, e)
        self._rebuild(e, members)
        return True

    def _rebuild(self, epoch: int, members: List[int]) -> None:
        """Fresh process group, communicators, step control and live server
        over ``members`` (original ranks), in this same process; the model's
        weights are kept. Requests that reach the old servable meanwhile fail
        UNAVAILABLE; the registry swaps in the new one at the end."""
        old_sched, old_eng = self.sched, self.engine
        try:
            old_eng.abort()  # the old communicators: nobody waits on a dead peer
        except Exception:  # noqa: BLE001
            log.exception("communicator abort failed")
        old_sched.close()  # launcher / completer drain (failed steps answer UNAVAILABLE)
        if dist.is_initialized():
            dist.destroy_process_group()
        world, rank = len(members), members.index(self.orig_rank)
        if world > 1:
            # control plane only (gloo): the data path is the native communicators
            dist.init_process_group("gloo", store=dist.PrefixStore(f"dtfs/pg/{epoch}", self._store), rank=rank,
                                    world_size=world,
                                    timeout=datetime.timedelta(seconds=max(60.0, self.cfg.serving.step_timeout_s)))
        ctx = DistContext(rank=rank, world=world, local_rank=self.ctx.local_rank, device=self.ctx.device,
                          backend="gloo" if world > 1 else "none")
        self.epoch, self.members = epoch, list(members)
        self._injected_comm_error = None
        self._build(ctx, first=False, store=self._store, model=old_eng.ex.model)
        args = getattr(self, "_native_front_args", None)
        if args is not None and self.serves and self.front is not None:
            # the native front door is bound to one live server: re-open it
            # over the new one (clients see a short UNAVAILABLE window)
            old_front = self.front
            old_front.stop()
            from .native_front import NativeGrpcFront

            self.front = NativeGrpcFront(self.service, self.sched, port=args[0], host=args[1], threads=args[2]).start()
        self.recoveries += 1
        log.warning("rank %d serving again as rank %d of %d (epoch %d)", self.orig_rank, rank, world, epoch)

    # -- front door ---------------------------------------------------------------------
    def start_grpc(self, port: int = 9999, host: str = "0.0.0.0", max_workers: int = 32,
                   monitoring_port: Optional[int] = None) -> int:
        """monitoring_port: also serve Prometheus metrics (serving/monitoring.py)."""
        from .grpc_server import GrpcFrontDoor
        from .monitoring import ServingMetrics

        assert self.serves, "this rank is not a front door"
        self.metrics = ServingMetrics(self.registry)
        self.front = GrpcFrontDoor(self.service, port=port, host=host, max_workers=max_workers,
                                   metrics=self.metrics).start()
        if monitoring_port is not None:
            self.metrics.serve_http(monitoring_port, host)
        return self.front.port

    def start_native_grpc(self, port: int = 9999, host: str = "0.0.0.0", threads: int = 4) -> int:
        """The C++ h2c front door (serving/native_front.py) over this rank's
        live server; a rebuilt cluster re-opens it over the new one."""
        from .native_front import NativeGrpcFront

        assert self.serves, "this rank is not a front door"
        with self._lock:
            self._native_front_args = (port, host, threads)
            self.front = NativeGrpcFront(self.service, self.sched, port=port, host=host, threads=threads).start()
            return self.front.port

    # -- followers ----------------------------------------------------------------------
    def serve_follower(self) -> int:
        """A rank without a front door: its live server joins every step the
        front door proposes. Returns the steps served once the front door
        stops the cluster; raises when the cluster breaks."""
        if self.ctl is None:
            return 0
        fault_after = int(self.follower_fault.get("after", -1))
        while True:
            ctl, sched = self.ctl, self.sched
            if ctl is None:  # rebuilt as a one-rank cluster (nothing to follow)
                return sched.stats()["steps"]
            if fault_after >= 0:
                if sched.stats()["steps"] >= fault_after:
                    log.error("fault injection: follower rank %d exits after %d steps", self.rank, fault_after)
                    os._exit(int(self.follower_fault.get("code", 17)))
                ctl.wait_event(0.002)
            else:
                ctl.wait_event(1.0)
            if ctl.stop_requested:
                steps = sched.stats()["steps"]
                sched.close()
                return steps
            if ctl.broken_by >= 0 or sched.broken or ctl.epoch > 0:
                if self.recover_on and self._recover():
                    continue
                raise RuntimeError(f"cluster broken: {self.broken or f'rank {ctl.broken_by} gave up'}")

    # -- shutdown ---------------------------------------------------------------------------
    def stop(self) -> None:
        self._stopping.set()
        if self.metrics is not None:
            self.metrics.stop()
        if self.front is not None:
            self.front.stop()
            self.front = None
        if self.ctl is not None and self.rank == 0:
            self.ctl.request_stop()  # followers close their live servers too
        if self.registry is not None:
            # drains this rank's live server (every launched step completes),
            # then stops the replica-cache refresher and unmaps the peers'
            # stores (LiveScheduler.close -> ShardedDLRM.release)
            self.registry.close()
        elif self.sched is not None:
            self.sched.close()
        wd = getattr(self, "_watchdog", None)
        if wd is not None and wd is not threading.current_thread():
            wd.join(timeout=10)


def main(argv=None):
    ap = argparse.ArgumentParser(description="multi-GPU CTR model server (rank 0 = PredictionService front door)")
    ap.add_argument("--preset", default="deepfm_fanout4")
    ap.add_argument("--mode", default="scatter", choices=["scatter", "alltoall", "local"],
                    help="scatter: rank 0 is the only front door; alltoall: every rank serves on port + rank; "
                         "local: every rank serves its own requests on port + rank (sharded DLRM: tables read "
                         "where they live, config 4)")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--grpc-workers", type=int, default=32)
    ap.add_argument("--front", default="native", choices=["native", "grpcio"],
                    help="native: C++ h2c front door, Predict straight into the live server; grpcio: Python gRPC")
    ap.add_argument("--front-threads", type=int, default=4, help="native front door: event-loop threads")
    ap.add_argument("--monitoring-port", type=int, default=None,
                    help="serve Prometheus metrics over HTTP on this port (rank 0)")
    ap.add_argument("--control-timeout-s", type=float, default=5.0,
                    help="a rank silent (no heartbeat) this long breaks the cluster")
    ap.add_argument("--step-timeout-s", type=float, default=30.0,
                    help="a GPU step not finished this long breaks the cluster (UNAVAILABLE)")
    ap.add_argument("--recover", action="store_true",
                    help="after a rank dies, rebuild the cluster over the survivors and keep serving")
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
                        step_timeout_s=a.step_timeout_s, mode=a.mode, recover=a.recover)
    rc = 0
    try:
        if not a.no_gc_freeze:  # every rank, after warm-up, before traffic
            tune_for_serving()
        if srv.serves:
            p = a.port + (srv.rank if a.mode in ("alltoall", "local") else 0)
            if a.front == "native":
                port = srv.start_native_grpc(p, a.host, a.front_threads)
                if a.monitoring_port is not None and srv.rank == 0:
                    from .monitoring import ServingMetrics

                    srv.metrics = ServingMetrics(srv.registry)
                    srv.metrics.serve_http(a.monitoring_port, a.host)
            else:
                port = srv.start_grpc(p, a.host, a.grpc_workers, a.monitoring_port if srv.rank == 0 else None)
            print(f"rank {srv.rank}: serving on port {port} over {ctx.world} GPU(s) ({a.mode}, {a.front} front door)",
                  flush=True)
            stop = threading.Event()

            def on_term(*_):
                stop.set()
                if srv.front:
                    srv.front.stop()

            signal.signal(signal.SIGTERM, on_term)
            try:
                while True:  # a rebuilt cluster swaps in a new native front door
                    f = srv.front
                    f.wait()
                    if stop.is_set() or srv.front is f:
                        break
            except KeyboardInterrupt:
                pass
        else:
            srv.serve_follower()
    except Exception:  # noqa: BLE001 - a follower that lost its peers
        log.exception("rank %d failed", srv.rank)
        rc = 3
    finally:
        srv.stop()
        if rc == 0:
            shutdown()
    return rc


if __name__ == "__main__":
    raise SystemExit(main())

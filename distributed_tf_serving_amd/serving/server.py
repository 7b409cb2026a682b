"""ModelServer: the TF-Serving ModelServer equivalent for one GPU (or CPU).

Builds a servable per configured model (random-init weights of the configured
architecture), captures its HIP graphs for every batch bucket, starts its
batching scheduler, and serves the PredictionService in-process and/or over
gRPC::

    python -m distributed_tf_serving_amd.serving.server --preset deepfm_1gpu --port 9999
    python -m distributed_tf_serving_amd.serving.server --preset wdl_tiny_cpu --port 9999 --device cpu
"""
from __future__ import annotations

import argparse
import logging
import signal
from typing import Optional

import torch

from ..config import Config, load_preset
from ..models import build_model
from ..parallel.dist import DistContext
from ..parallel.fanout import FanoutEngine
from ..utils.gc_tuning import tune_for_serving
from .arena import ArenaLayout
from .batching import BatchingScheduler
from .executor import ShardExecutor
from .live import LiveScheduler
from .monitoring import ServingMetrics
from .packing import PackedLayout, layout_for
from .registry import ModelRegistry, Servable, Signature
from .service import PredictionServiceImpl

log = logging.getLogger(__name__)


def pick_device(pref: str = "auto") -> torch.device:
    if pref == "cpu" or (pref == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    if pref.startswith("cuda") and ":" in pref:
        return torch.device(pref)
    return torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)


def live_enabled(cfg: Config, device: torch.device) -> bool:
    """Servables run on the native live server: a CPU model (Python forward
    behind the C++ core), or a GPU model whose step replays captured graphs."""
    sc = cfg.serving
    return bool(sc.live) and (device.type != "cuda" or sc.use_graphs)


def build_engine(cfg: Config, device=None, slots: int = 3, ctx: Optional[DistContext] = None,
                 mode: str = "local", group=None, model=None, scatter_tag: str = "serve",
                 store=None) -> FanoutEngine:
    """Model + executor + fan-out engine of one rank, every bucket prepared
    (HIP graphs captured). With ``ctx`` of a multi-rank job, DLRM tables are
    sharded over the ranks (parallel/embedding_sharding.py) and ``mode``
    scatter / alltoall fans every batch out over the ranks. A servable of the
    live server ingests request arenas (the GPU unpacks raw request bytes).
    ``group``: process group of the step's collectives (CPU: a dedicated gloo
    group, since they run on the live server's launcher thread). ``model``:
    reuse a built replica (a cluster rebuilt over fewer ranks keeps its weights).
    ``scatter_tag``: store prefix of the shared-scatter segment (unique per
    segment: a rebuilt cluster makes a new one)."""
    from ..parallel.embedding_sharding import build_parallel_model

    sc = cfg.serving
    dev = torch.device(device) if device is not None else (ctx.device if ctx is not None else pick_device(sc.device))
    ctx = ctx or DistContext(device=dev)
    sharded = getattr(getattr(model, "plan", None), "world", 1) > 1
    if model is None or sharded or getattr(model, "has_collectives", False):
        # sharded tables re-shard over the new world
        if model is not None and hasattr(model, "stop_cache"):
            model.stop_cache()
        model = build_parallel_model(cfg.model, dev, ctx, group=group)
    world = ctx.world if ctx.is_distributed else 1
    buckets = sorted(set(sc.allowed_batch_sizes) | {sc.max_batch_rows})
    if mode == "alltoall" and world > 1:  # every rank's rows split evenly over the GPUs
        buckets = [b for b in buckets if b % world == 0] or [sc.max_batch_rows * world]
    use_graphs = sc.use_graphs
    live = live_enabled(cfg, dev)
    # scatter on one node through rank 0's shared arenas: the step is local
    shared = live and mode == "scatter" and world > 1 and getattr(sc, "scatter_path", "shared") == "shared"
    # rows exchanged between GPUs travel narrow (int32 rows + fp32 weights)
    fanout = live and mode != "local" and world > 1 and not shared
    layout = layout_for(cfg.model, fanout) if fanout else PackedLayout(cfg.model.num_fields)
    ex = ShardExecutor(model, layout, buckets, dev, use_graphs=use_graphs, slots=slots)
    if live:
        rows_in = max(buckets) * (world if mode == "scatter" else 1)
        # shared scatter: shares are cut from the row table, so ids are decoded on the host
        arena = ArenaLayout(cfg.model.num_fields, max_rows=rows_in, gpu_varint=not shared)
        seg = None
        if shared:
            from ..parallel.shared_scatter import live_narrowing, scatter_for_engine

            nm, nw = live_narrowing(model, dev.type == "cuda", bool(getattr(sc, "narrow_ingest", True)))
            seg = scatter_for_engine(ctx, cfg.model.num_fields, arena.capacity, slots, max(buckets),
                                     tag=scatter_tag, store=store, narrow_modulo=nm, narrow_wts_cols=nw)
        eng = FanoutEngine(ex, ctx, mode=mode, ingest="arena", group=group, arena=arena, shared_scatter=seg)
    else:
        eng = FanoutEngine(ex, ctx, mode=mode, group=group)
    for B in buckets:
        eng.prepare(B)
    if hasattr(model, "start_cache"):  # peer exchange: keep the hot-row replica current
        model.start_cache(getattr(sc, "hot_cache_refresh_s", 1.0))
    return eng


def build_servable(cfg: Config, device=None, version: Optional[int] = None, slots: int = 3,
                   engine: Optional[FanoutEngine] = None, control=None, liveness_only: bool = False) -> Servable:
    """``control``: the job's StepControl (parallel/control.py) when the
    engine's step has collectives (every rank's live server agrees on it), or
    with ``liveness_only`` for ranks that serve independently but read each
    other's memory (heartbeats + broken flag only)."""
    sc = cfg.serving
    eng = engine or build_engine(cfg, device, slots)
    model = eng.ex.model
    world = eng.world if eng.mode == "scatter" else 1
    if eng.ingest == "arena":
        if eng.lockstep and eng.world > 1 and control is None:
            raise ValueError("a multi-rank engine with collectives in its step needs a StepControl")
        sched = LiveScheduler(eng, sc, version=sc.version if version is None else version,
                              step_timeout_s=sc.step_timeout_s, control=control,
                              peer_timeout_s=getattr(sc, "peer_timeout_s", 5.0), start_paused=control is not None,
                              liveness_only=liveness_only)
    else:
        sched = BatchingScheduler(eng, max_batch_rows=sc.max_batch_rows, batch_timeout_us=sc.batch_timeout_us,
                                  max_queued_rows=sc.max_queued_rows, depth=max(1, slots - 1), name=sc.model_name,
                                  fanout_world=world, max_request_rows=sc.max_request_rows)
    sig = model.signature()
    sigs = {sc.signature_name: Signature(inputs=sig["inputs"], outputs=sig["outputs"], method_name=sig["method_name"])}
    return Servable(name=sc.model_name, version=sc.version if version is None else version, model=model,
                    scheduler=sched, signatures=sigs, ids_key=sc.ids_key, wts_key=sc.wts_key,
                    output_key=sc.output_key, fields=cfg.model.num_fields)


class ModelServer:
    def __init__(self, cfg: Config, device=None):
        self.cfg = cfg
        self.registry = ModelRegistry()
        self.registry.load(build_servable(cfg, device))
        self.service = PredictionServiceImpl(self.registry, cfg.serving.request_timeout_s)
        self.metrics = ServingMetrics(self.registry)
        self.front = None

    def start_grpc(self, port: int = 9999, host: str = "0.0.0.0", max_workers: int = 32):
        from .grpc_server import GrpcFrontDoor

        self.front = GrpcFrontDoor(self.service, port=port, host=host, max_workers=max_workers,
                                   metrics=self.metrics).start()
        return self.front.port

    def start_native_grpc(self, port: int = 9999, host: str = "0.0.0.0", threads: int = 4) -> int:
        """The C++ h2c front door (serving/native_front.py): Predict goes from
        the event loop straight into the servable's native live server."""
        from .live import LiveScheduler
        from .native_front import NativeGrpcFront

        sched = self.registry.resolve(self.cfg.serving.model_name).scheduler
        if not isinstance(sched, LiveScheduler):
            raise ValueError("the native front door needs a live-server servable (serving.live)")
        self.front = NativeGrpcFront(self.service, sched, port=port, host=host, threads=threads).start()
        return self.front.port

    def start_monitoring(self, port: int, host: str = "0.0.0.0") -> int:
        """Prometheus text format over HTTP (TF-Serving's monitoring endpoint)."""
        return self.metrics.serve_http(port, host)

    def stop(self) -> None:
        self.metrics.stop()
        if self.front is not None:
            self.front.stop()
            self.front = None
        self.registry.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def main(argv=None):
    ap = argparse.ArgumentParser(description="MI355X CTR model server (TF-Serving PredictionService)")
    ap.add_argument("--preset", default="deepfm_1gpu")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--device", default=None)
    ap.add_argument("--model-name", default=None)
    ap.add_argument("--grpc-workers", type=int, default=32)
    ap.add_argument("--monitoring-port", type=int, default=None,
                    help="serve Prometheus metrics over HTTP on this port (TF-Serving monitoring endpoint)")
    ap.add_argument("--inject-fault", default="",
                    help="failure testing, e.g. 'after:100,kind:error' (serving/faults.py)")
    ap.add_argument("--no-gc-freeze", action="store_true",
                    help="leave CPython's cyclic GC at its defaults (utils/gc_tuning.py)")
    ap.add_argument("--frontends", type=int, default=1,
                    help="server processes sharing the port (SO_REUSEPORT), each with its own model replica and "
                         "live server on the same GPU: scales the grpcio front door past one GIL "
                         "(profiles/grpc_ceiling.md)")
    ap.add_argument("--frontend-index", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--front", default="auto", choices=["auto", "native", "grpcio"],
                    help="native: C++ h2c front door, Predict straight into the live server (csrc/net); grpcio: "
                         "the Python gRPC server; auto: native when the servable runs on the live server and no "
                         "fault is injected")
    ap.add_argument("--front-threads", type=int, default=4, help="native front door: event-loop threads")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    children = []
    if a.frontends > 1 and a.frontend_index == 0:
        # started before this process touches the GPU; each child is a full server
        import subprocess
        import sys

        base = [x for x in (argv if argv is not None else sys.argv[1:])]
        for i in range(1, a.frontends):
            extra = ["--frontends", "1", "--frontend-index", str(i)]
            args = [x for x in base]
            if "--monitoring-port" in args:  # only frontend 0 serves metrics
                j = args.index("--monitoring-port")
                del args[j:j + 2]
            children.append(subprocess.Popen([sys.executable, "-m", "distributed_tf_serving_amd.serving.server",
                                              *args, *extra]))
    cfg = load_preset(a.preset)
    if a.model_name:
        cfg.serving.model_name = a.model_name
    srv = ModelServer(cfg, device=a.device)
    if a.inject_fault:
        from .faults import FaultInjector, FaultSpec, FaultyService

        srv.service = FaultyService(srv.service, FaultInjector(FaultSpec.parse(a.inject_fault)))
    if not a.no_gc_freeze:  # after warm-up (graphs captured), before the port takes traffic
        logging.getLogger(__name__).info("gc: %s", tune_for_serving())
    from .live import LiveScheduler

    live = isinstance(srv.registry.resolve(cfg.serving.model_name).scheduler, LiveScheduler)
    front = a.front if a.front != "auto" else ("native" if live and not a.inject_fault else "grpcio")
    if front == "native":
        port = srv.start_native_grpc(a.port, a.host, a.front_threads)
    else:
        port = srv.start_grpc(a.port, a.host, a.grpc_workers)
    if a.monitoring_port is not None:
        srv.start_monitoring(a.monitoring_port, a.host)
    if a.frontend_index == 0:
        print(f"serving model {cfg.serving.model_name!r} ({cfg.model.family}) on port {port} ({front} front door)"
              + (f" ({a.frontends} frontend processes)" if a.frontends > 1 else ""), flush=True)
    signal.signal(signal.SIGTERM, lambda *_: srv.stop())
    try:
        srv.front.wait()
    except KeyboardInterrupt:
        pass
    finally:
        srv.stop()
        for c in children:
            c.terminate()
        for c in children:
            try:
                c.wait(timeout=30)
            except Exception:  # noqa: BLE001
                c.kill()


if __name__ == "__main__":
    main()

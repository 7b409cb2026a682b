"""Prometheus metrics for the model server (TF-Serving's monitoring endpoint).

TF-Serving exposes its request / batching metrics in the Prometheus text
format when started with a monitoring config (``prometheus_config { enable:
true path: "/monitoring/prometheus/metrics" }``). The reference client never
reads them (it only prints per-request latency,
DCNClient.java:198-202), but a user switching servers expects the endpoint.

``ServingMetrics`` keeps its own ``CollectorRegistry`` (no global state, so
several servers in one process - tests - do not collide):

* ``:tensorflow:serving:request_count{API,status}`` - every RPC by outcome
  (``OK`` or the gRPC status name), counted in the gRPC front door;
* ``:tensorflow:serving:request_latency{API}`` - RPC wall time histogram (us);
* per servable, read from the batching scheduler at scrape time
  (serving/batching.py ``stats``): submitted / rejected / expired requests,
  batches (full / timeout), rows batched and served, GPU steps, and the
  average batch fill.
"""
from __future__ import annotations

import time
from typing import Optional

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest, start_http_server
from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily

from .registry import ModelRegistry

PREFIX = ":tensorflow:serving:"
DEFAULT_PATH = "/monitoring/prometheus/metrics"
# us buckets: the serving step is ~0.2-1 ms on an MI355X, gRPC adds ~1-3 ms
_LAT_BUCKETS = (50, 100, 200, 500, 1000, 2000, 5000, 10000, 20000, 50000, 100000, 500000, float("inf"))

# scheduler stats key -> (metric suffix, help, counter?)
_SCHED = {
    "submitted": ("batching_submitted", "requests submitted to the batching queue", True),
    "rejected": ("batching_rejected", "requests rejected by queue back-pressure", True),
    "expired": ("batching_expired", "requests dropped because their deadline passed in the queue", True),
    "batches": ("batching_batches", "batches formed", True),
    "full_batches": ("batching_full_batches", "batches closed because they were full", True),
    "timeout_batches": ("batching_timeout_batches", "batches closed by the batch timeout", True),
    "batched_rows": ("batching_rows", "candidate rows batched", True),
    "steps": ("gpu_steps", "serving steps completed on the device", True),
    "rows_served": ("rows_served", "candidate rows scored", True),
    # peer-exchange DLRM: the hot-row replica cache (hits / misses of the counted candidates)
    "hot_cache_rows": ("hot_cache_rows", "remote table rows held in this rank's replica cache", False),
    "hot_cache_refreshes": ("hot_cache_refreshes", "replica cache refreshes", True),
    "hot_cache_hits": ("hot_cache_hits", "counted remote lookups served by the replica cache", True),
    "hot_cache_misses": ("hot_cache_misses", "counted remote lookups read from the owner's HBM", True),
    "hot_cache_refresh_failures": ("hot_cache_refresh_failures", "replica cache refreshes that failed (retried)", True),
    "hot_cache_refresher_alive": ("hot_cache_refresher_alive", "1 while the replica cache refresher thread runs", False),
}


class _SchedulerCollector:
    """Scrape-time view of every loaded servable's batching scheduler."""

    def __init__(self, registry: ModelRegistry):
        self.registry = registry

    def collect(self):
        fams = {k: (CounterMetricFamily if c else GaugeMetricFamily)(PREFIX + name, doc,
                                                                       labels=["model_name", "version"])
                for k, (name, doc, c) in _SCHED.items()}
        fill = GaugeMetricFamily(PREFIX + "batching_avg_batch_rows", "average rows per batch",
                                 labels=["model_name", "version"])
        for name in self.registry.names():
            for v in self.registry.versions(name):
                try:
                    st = self.registry.resolve(name, v).scheduler.stats()
                except Exception:  # noqa: BLE001 - a servable being unloaded
                    continue
                labels = [name, str(v)]
                for k, fam in fams.items():
                    if k in st:
                        fam.add_metric(labels, float(st[k]))
                if st.get("batches"):
                    fill.add_metric(labels, st.get("batched_rows", 0) / st["batches"])
        yield from fams.values()
        yield fill


class ServingMetrics:
    def __init__(self, registry: Optional[ModelRegistry] = None):
        self.prom = CollectorRegistry()
        self.requests = Counter(PREFIX + "request_count", "RPCs by API and outcome", ["API", "status"],
                                registry=self.prom)
        self.latency = Histogram(PREFIX + "request_latency", "RPC latency in microseconds", ["API"],
                                 buckets=_LAT_BUCKETS, registry=self.prom)
        if registry is not None:
            self.prom.register(_SchedulerCollector(registry))
        self._http = None

    def observe(self, api: str, status: str, t0: float) -> None:
        """Record one RPC that started at ``time.perf_counter()`` value t0."""
        self.requests.labels(api, status).inc()
        self.latency.labels(api).observe((time.perf_counter() - t0) * 1e6)

    def exposition(self) -> bytes:
        return generate_latest(self.prom)

    def serve_http(self, port: int, addr: str = "0.0.0.0") -> int:
        """Serve the text format over HTTP (any path, incl. DEFAULT_PATH)."""
        server, _ = start_http_server(port, addr=addr, registry=self.prom)
        self._http = server
        return server.server_port

    def stop(self) -> None:
        if self._http is not None:
            self._http.shutdown()
            self._http.server_close()
            self._http = None

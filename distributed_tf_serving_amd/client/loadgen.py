"""Load generator: the reference DCNClient.main, with its knobs as flags.

Closed loop (reference mode): ``--concurrency`` threads each issue
``--requests`` back-to-back fan-out requests of ``--candidates`` candidates
split over the backends (reference DCNClient.java:205-241). Open loop:
``--qps`` issues requests on a fixed schedule and measures latency at that
offered load (BASELINE.json's "p50 request latency at fixed QPS").

Prints the reference's two line formats (keep them diff-able,
DCNClient.java:201-202, 235-236)::

    Thread <name>. Time cost with <n> is <ms> ms
    Average time cost with <C> is <ms> ms with <k> requests

plus one JSON summary line (p50/p90/p99/p999, QPS, CTR scores/s).

Backends: ``--hosts h1:9999,h2:9999`` (gRPC, ours or TF-Serving) or
``--inproc-preset wdl_tiny_cpu`` (start servers in this process).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import threading
import time
from typing import List, Optional

import numpy as np
import torch

from ..config import add_client_args, client_from_args
from .backends import GrpcBackend, InProcessBackend
from .fanout_client import FanoutClient, RequestSpec
from .synth import SyntheticRequests
from ..utils.gc_tuning import tune_for_serving


def percentile(xs: List[float], p: float) -> float:
    return float(np.percentile(np.asarray(xs), p)) if xs else float("nan")


def summarize(lat_ms: List[float], wall_s: float, candidates: int, errors: int = 0) -> dict:
    n = len(lat_ms)
    return {
        "requests": n,
        "errors": errors,
        "avg_ms": statistics.fmean(lat_ms) if lat_ms else None,
        "p50_ms": percentile(lat_ms, 50),
        "p90_ms": percentile(lat_ms, 90),
        "p99_ms": percentile(lat_ms, 99),
        "p999_ms": percentile(lat_ms, 99.9),
        "qps": n / wall_s if wall_s > 0 else None,
        "scores_per_s": n * candidates / wall_s if wall_s > 0 else None,
        "wall_s": wall_s,
    }


class LoadGenerator:
    def __init__(self, client: FanoutClient, candidates: int, fields: int = 43, id_mode: str = "reference",
                 id_space: int = 1_000_000, seed: int = 0, verbose: bool = True, out=sys.stdout):
        self.client = client
        self.candidates = candidates
        self.synth = SyntheticRequests(fields=fields, id_space=id_space, dist=id_mode, seed=seed)
        # like the reference, features are generated once, outside the timed region (DCNClient.java:209-210)
        ids, wts = self.synth.arrays(candidates)
        self.ids, self.wts = torch.from_numpy(ids), torch.from_numpy(wts)
        self.verbose = verbose
        self.out = out
        self.lat_ms: List[float] = []
        self.errors = 0
        self._lock = threading.Lock()

    def one(self) -> Optional[float]:
        t0 = time.perf_counter()
        try:
            res = self.client.predict(self.ids, self.wts)
        except Exception as e:  # noqa: BLE001
            with self._lock:
                self.errors += 1
            print(f"request failed: {e}", file=sys.stderr)
            return None
        ms = (time.perf_counter() - t0) * 1e3
        n = res.scores.numel()
        with self._lock:
            self.lat_ms.append(ms)
        if self.verbose:
            print(f"Thread {threading.current_thread().name}. Time cost with {n} is {ms} ms", file=self.out)
        return ms

    def closed_loop(self, concurrency: int, requests: int, warmup: int = 0) -> dict:
        for _ in range(warmup):
            self.one()
        self.lat_ms.clear()
        self.errors = 0

        def worker():
            for _ in range(requests):
                self.one()

        ths = [threading.Thread(target=worker, name=f"Thread-{i}") for i in range(concurrency)]
        t0 = time.perf_counter()
        [t.start() for t in ths]
        [t.join() for t in ths]
        wall = time.perf_counter() - t0
        if self.lat_ms:
            avg = sum(self.lat_ms) / len(self.lat_ms)
            print(f"Average time cost with {self.candidates} is {avg} ms with {len(self.lat_ms)} requests",
                  file=self.out)
        return summarize(self.lat_ms, wall, self.candidates, self.errors)

    def open_loop(self, qps: float, total: int, warmup: int = 0) -> dict:
        for _ in range(warmup):
            self.one()
        self.lat_ms.clear()
        self.errors = 0
        period = 1.0 / qps
        futs = []
        t0 = time.perf_counter()
        for i in range(total):
            target = t0 + i * period
            d = target - time.perf_counter()
            if d > 0:
                time.sleep(d)
            t_issue = time.perf_counter()
            f = self.client.predict_async(self.ids, self.wts)
            f.add_done_callback(lambda f, t=t_issue: self._record_async(f, t))
            futs.append(f)
        for f in futs:
            try:
                f.result()
            except Exception:  # noqa: BLE001
                pass
        wall = time.perf_counter() - t0
        return summarize(self.lat_ms, wall, self.candidates, self.errors)

    def _record_async(self, f, t_issue):
        with self._lock:
            if f.exception() is None:
                self.lat_ms.append((time.perf_counter() - t_issue) * 1e3)
            else:
                self.errors += 1


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_client_args(ap)
    ap.add_argument("--inproc-preset", default=None, help="start N in-process servers with this preset")
    ap.add_argument("--quiet", action="store_true", help="suppress per-request lines")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-gc-freeze", action="store_true", help="leave CPython's cyclic GC at its defaults")
    a = ap.parse_args(argv)
    c = client_from_args(a)
    servers = []
    if a.inproc_preset:
        from ..config import load_preset
        from ..serving.server import ModelServer

        cfg = load_preset(a.inproc_preset)
        cfg.serving.model_name = c.model_name
        servers = [ModelServer(cfg) for _ in range(c.backends)]
        backends = [InProcessBackend(s.service, name=f"inproc{i}") for i, s in enumerate(servers)]
    else:
        hosts = c.hosts if a.hosts else ["127.0.0.1"] * c.backends
        backends = [GrpcBackend(h if ":" in h else f"{h}:{c.port}") for h in hosts]
    spec = RequestSpec(model_name=c.model_name, signature_name=c.signature_name, output_key=c.output_key,
                       raw=c.raw_tensors)
    client = FanoutClient(backends, spec, pool_threads=c.pool_threads, full_async=c.full_async,
                          sort_scores=c.sort_scores, timeout_s=c.deadline_s or None)
    lg = LoadGenerator(client, c.candidates, fields=c.fields, id_mode=c.id_mode, id_space=c.id_space, seed=c.seed,
                       verbose=not a.quiet)
    if not a.no_gc_freeze:
        tune_for_serving()  # a GC pause in the load generator is client-side latency, not the server's
    try:
        if c.qps > 0:
            summary = lg.open_loop(c.qps, c.requests * c.concurrency, warmup=c.warmup)
            summary["mode"] = f"open-loop {c.qps} qps"
        else:
            summary = lg.closed_loop(c.concurrency, c.requests, warmup=c.warmup)
            summary["mode"] = f"closed-loop x{c.concurrency}"
        summary.update(backends=len(backends), candidates=c.candidates, full_async=c.full_async)
        print(json.dumps(summary), flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(summary, f)
    finally:
        client.close()
        for s in servers:
            s.stop()


if __name__ == "__main__":
    main()

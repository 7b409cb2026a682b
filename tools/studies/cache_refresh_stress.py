"""Replica-cache refreshes racing cached lookups in ONE process (the served
2-rank DLRM run stalled its steps once the background refresher ran every
50 ms): a PeerTables over two local stores, a large HotRowCache learned from
Zipf lookups, then one thread launching cached lookups back to back on its own
stream while the main thread refreshes every --period seconds. Reports each
refresh's time and the worst lookup batch; exits 2 if a batch stalls > 10 s.

    python -m tools.studies.cache_refresh_stress [--cap 67108864] [--period 0.05]
"""
from __future__ import annotations

import argparse
import json
import os
import threading
import time

import numpy as np
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.parallel.hot_cache import HotRowCache, PeerTables


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tables", type=int, default=30)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--cap", type=int, default=1 << 26)
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--period", type=float, default=0.05)
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--nbatches", type=int, default=8)
    ap.add_argument("--dist", default="zipf", choices=["zipf", "uniform"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    T, R = a.tables, a.rows
    stores = [torch.zeros(T * R, 64, dtype=torch.bfloat16, device=dev) for _ in range(2)]
    owner = [t % 2 for t in range(T)]
    p = PeerTables(stores, owner, [t * R for t in range(T)], [R] * T, rank=0)
    c = HotRowCache(p, capacity=a.cap)
    rng = np.random.default_rng(1)
    def draw():
        if a.dist == "uniform":
            return rng.integers(0, R, (a.batch, T))
        return np.minimum(rng.zipf(1.1, (a.batch, T)), R) - 1

    batches = [torch.from_numpy(draw()).to(dev) for _ in range(a.nbatches)]
    dense = torch.randn(a.batch, 64, device=dev).to(torch.bfloat16)
    # learn: every candidate's remote keys sampled
    c.set_sample_period(1)
    for i in range(4):
        for b in batches:
            ops.dot_interaction_gather_peer(dense, b, p, c)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c.refresh()
        print(json.dumps({"learn_refresh": i, "ms": round((time.perf_counter() - t0) * 1e3, 2),
                          "hot_rows": int(c.keys.numel())}), flush=True)
    c.set_sample_period(0)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    c.set_step_stream(s.cuda_stream)
    stop = threading.Event()
    stats = {"batches": 0, "worst_ms": 0.0}

    def worker():
        k = 0
        with torch.cuda.stream(s):
            while not stop.is_set():
                t0 = time.perf_counter()
                for _ in range(4):
                    ops.dot_interaction_gather_peer(dense, batches[k % len(batches)], p, c)
                    k += 1
                s.synchronize()
                dt = (time.perf_counter() - t0) * 1e3
                stats["batches"] += 4
                stats["worst_ms"] = max(stats["worst_ms"], dt)

    th = threading.Thread(target=worker, daemon=True)
    th.start()
    times = []
    t_end = time.perf_counter() + a.seconds
    last = time.perf_counter()
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        c.refresh()
        times.append((time.perf_counter() - t0) * 1e3)
        if time.perf_counter() - last > 1.0:
            last = time.perf_counter()
            print(json.dumps({"refreshes": len(times), "lookup_batches": stats["batches"],
                              "worst_batch_ms": round(stats["worst_ms"], 1)}), flush=True)
        if stats["worst_ms"] > 10000:
            print("lookup stalled > 10 s", flush=True)
            os._exit(2)
        time.sleep(a.period)
    stop.set()
    th.join(timeout=30)
    if th.is_alive():
        print("lookup thread stuck", flush=True)
        os._exit(2)
    print(json.dumps({"refreshes": len(times), "refresh_ms_median": round(float(np.median(times)), 2),
                      "refresh_ms_max": round(max(times), 2), "lookup_batches": stats["batches"],
                      "worst_batch_ms": round(stats["worst_ms"], 1)}), flush=True)


if __name__ == "__main__":
    main()

"""Step cost per padding bucket (the server's allowed_batch_sizes): for each
bucket, the serial latency of one full step (H2D of a filled request arena ->
captured step -> scores on the host) and the pipelined time per step with
every slot in flight. Tells which small buckets are worth having: a bucket
whose step costs nearly as much as the next larger one only adds queueing
under load (bench.py --small-buckets).

    python -m tools.studies.bucket_cost --buckets 512,1024,2048,4096,8192,16384
"""
from __future__ import annotations

import argparse
import json
import statistics
import time

import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.parallel.dist import DistContext
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine
from distributed_tf_serving_amd.serving.arena import ArenaLayout
from distributed_tf_serving_amd.serving.executor import ShardExecutor
from distributed_tf_serving_amd.serving.packing import PackedLayout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--family", default="deepfm")
    ap.add_argument("--buckets", default="512,1024,2048,4096,8192,16384")
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--slots", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = ModelConfig(family=a.family)
    model = build_model(cfg, dev)
    F = cfg.num_fields
    buckets = [int(x) for x in a.buckets.split(",")]
    ex = ShardExecutor(model, PackedLayout(F), buckets, dev, slots=a.slots)
    AL = ArenaLayout(F, max_rows=max(buckets))
    eng = FanoutEngine(ex, DistContext(device=dev), mode="local", ingest="arena", arena=AL)
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=3)
    out = []
    for B in buckets:
        eng.prepare(B)
        reqs = [synth.serialized(min(512, B), raw=True) for _ in range(max(1, B // 512))]
        arenas, used = [], []
        for s in range(a.slots):
            ar = eng.host_arena(s)
            ab = AL.build(ar, AL.place(ar, reqs))
            arenas.append(ar)
            used.append(ab.used_bytes)
        for _ in range(5):
            eng.launch(B, 0, src=arenas[0], nbytes=used[0]).wait()
        lat = []
        for i in range(a.iters):
            t0 = time.perf_counter()
            eng.launch(B, i % a.slots, src=arenas[i % a.slots], nbytes=used[i % a.slots]).wait()
            lat.append((time.perf_counter() - t0) * 1e6)
        hs = []
        t0 = time.perf_counter()
        for i in range(a.iters):
            if len(hs) == a.slots:
                hs.pop(0).wait()
            hs.append(eng.launch(B, i % a.slots, src=arenas[i % a.slots], nbytes=used[i % a.slots]))
        for h in hs:
            h.wait()
        pipe = (time.perf_counter() - t0) * 1e6 / a.iters
        r = {"bucket": B, "serial_p50_us": round(statistics.median(lat), 1), "pipelined_us_per_step": round(pipe, 1),
             "rows_per_us": round(B / pipe, 1)}
        out.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()

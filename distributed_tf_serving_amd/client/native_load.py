"""Native gRPC load generator: the reference client's closed loop
(reference DCNClient.java:205-241: ``--concurrency`` threads x ``--requests``
back-to-back Predicts of ``--candidates`` candidates) on C++ h2c clients
(csrc/net/h2_client.cpp), so an over-the-network measurement is not bounded by
a Python gRPC client. One connection per client thread; the requests are
built once, like the reference's (DCNClient.java:209-210), packed
``int64_val`` / ``float_val`` by default.

    python -m distributed_tf_serving_amd.client.native_load --port 9999 --candidates 1500 \\
        --concurrency 6 --requests 1000 --id-mode reference

Prints the reference's average line and one JSON summary (avg / p50 / p99,
requests/s, scores/s).
"""
from __future__ import annotations

import argparse
import json
import sys

import numpy as np
import torch

from ..ops import native
from .synth import SyntheticRequests

PREDICT = "/tensorflow.serving.PredictionService/Predict"


def build_requests(candidates: int, fields: int, id_mode: str, n: int, raw: bool, model: str = "DCN"):
    synth = SyntheticRequests(fields=fields, id_space=1 << 40, dist=id_mode, seed=7)
    out = []
    for _ in range(n):
        ids, wts = synth.arrays(candidates)
        out.append(native().encode_predict_request(model, "serving_default", None,
                                                   [("feat_ids", torch.from_numpy(ids)),
                                                    ("feat_wts", torch.from_numpy(wts))], raw))
    return out


def run(host: str, port: int, requests, concurrency: int, count: int, warmup: int, timeout_s: float,
        candidates: int) -> dict:
    r = native().run_grpc_load(host, port, PREDICT, requests, concurrency=concurrency, warmup=warmup, count=count,
                               timeout_s=timeout_s)
    lat = np.asarray(r["latency_us"], dtype=np.float64) * 1e-3
    win = r["window_us"] * 1e-6
    return {"requests": int(lat.size), "errors": int(r["errors"]), "first_error": r["first_error"] or None,
            "avg_ms": float(lat.mean()) if lat.size else None,
            "p50_ms": float(np.percentile(lat, 50)) if lat.size else None,
            "p99_ms": float(np.percentile(lat, 99)) if lat.size else None,
            "requests_per_s": round(lat.size / win, 1) if win > 0 else None,
            "scores_per_s": round(lat.size * candidates / win, 1) if win > 0 else None,
            "clients": concurrency, "candidates": candidates, "client": "native h2c (csrc/net/h2_client.cpp)"}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--candidates", type=int, default=1500)
    ap.add_argument("--fields", type=int, default=43)
    ap.add_argument("--concurrency", type=int, default=6)
    ap.add_argument("--requests", type=int, default=1000, help="per client thread (timed)")
    ap.add_argument("--warmup", type=int, default=10, help="per client thread (untimed)")
    ap.add_argument("--id-mode", default="reference", choices=["reference", "uniform", "zipf"])
    ap.add_argument("--raw", action="store_true", help="tensor_content instead of int64_val / float_val")
    ap.add_argument("--pool", type=int, default=16, help="distinct requests to cycle through")
    ap.add_argument("--timeout-s", type=float, default=30.0)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)
    reqs = build_requests(a.candidates, a.fields, a.id_mode, 1 if a.id_mode == "reference" else a.pool, a.raw)
    res = run(a.host, a.port, reqs, a.concurrency, a.concurrency * a.requests, a.concurrency * a.warmup,
              a.timeout_s, a.candidates)
    if res["avg_ms"] is not None:
        print(f"Average time cost with {a.candidates} is {res['avg_ms']} ms with {res['requests']} requests")
    print(json.dumps(res), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(res, f)
    return 0 if res["errors"] == 0 and res["requests"] > 0 else 1


if __name__ == "__main__":
    sys.exit(main())

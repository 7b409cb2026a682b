"""The one-launch DeepFM tower (csrc/kernels/gather_mlp.hip) against the
two-kernel form it replaces (one-wave gather-GEMM + MLP tail), interleaved, on
the served shapes: 1M x 64 table, 43 fields, 1024-512-256, Zipf ids over 2^40.
Both forms include the rows' resolve: the two-kernel form runs the resolve
pass (embed_resolve) first, the one-launch tower resolves in its prologue.

    python -m tools.studies.gather_mlp_study [--rows 8192,16384]
"""
from __future__ import annotations

import argparse
import json
import statistics

import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model


def _time(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="8192,16384")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = build_model(ModelConfig(family="deepfm", vocab_size=1_000_000), dev)
    l1, l2, l3 = m.mlp.layers
    for B in [int(x) for x in a.rows.split(",")]:
        ids, wts = SyntheticRequests(fields=43, id_space=1 << 40, dist="zipf", seed=B).arrays(B)
        ids, wts = torch.from_numpy(ids).to(dev), torch.from_numpy(wts).to(dev)
        out = torch.empty(B, dtype=torch.float32, device=dev)

        def one():
            return ops.gather_mlp(m.emb, ids, wts, m.lin, m.cfg.vocab_size, m.fm_bias, m.mlp.layers, m.head_w,
                                  m.head_b, fm=True, out=out)

        def two():
            h, parts = ops.embed_gemm(m.emb, ids, wts, m.lin, m.cfg.vocab_size, m.fm_bias, l1.weight, l1.bias, "relu",
                                      fm2=True, packed_w=lambda: l1.packed("32"))
            return ops.mlp_tail(h, l2.packed(), l2.bias, l2.act, l3.packed(), l3.bias, l3.act, m.head_w, m.head_b,
                                extra=parts, out=out)

        times = {"gather_mlp": [], "two_kernels": []}
        for _ in range(a.rounds):
            times["gather_mlp"].append(_time(one))
            times["two_kernels"].append(_time(two))
        y1 = one().clone()
        y2 = two().clone()
        torch.cuda.synchronize()
        res = {"rows": B, **{f"{k}_us": round(statistics.median(v), 2) for k, v in times.items()},
               "max_diff": float((y1 - y2).abs().max())}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Tile order of the DCN-v2 fp8 cross GEMM (csrc/kernels/gemm.hip
gemm_8ph_kernel, ``gm``): N-fastest (0) against groups of gm row tiles walked
M-fastest, interleaved rounds, one cross layer at the served shapes.

    python -m tools.studies.cross_order_study [--rows 8192,16384] [--gm 0,4,8,16]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics

import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.models import build_model


def _time(fn, iters=20):
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
    ap.add_argument("--gm", default="0,4,8,16")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = build_model(load_preset("dcn_v2_fp8").model, dev)
    gms = [int(x) for x in a.gm.split(",")]
    for B in [int(x) for x in a.rows.split(",")]:
        x0 = (torch.randn(B, m.d, device=dev) * 0.5).to(torch.bfloat16)
        q, sx = ops.quant_rows_fp8(x0, ops.FP8_K_PAD)
        layer = m.cross[1]

        def c8():
            return ops.cross_gemm_fp8(q, sx, layer.w_fp8, layer.w_scale, layer.bias, x0, x0, want_z=True)

        times = {g: [] for g in gms}
        outs = {}
        for _ in range(a.rounds):
            for g in gms:
                os.environ["DTFS_CROSS_GM"] = str(g)
                times[g].append(_time(c8))
        for g in gms:
            os.environ["DTFS_CROSS_GM"] = str(g)
            outs[g] = c8()[0].clone()
        torch.cuda.synchronize()
        base = outs[gms[0]]
        res = {"rows": B, **{f"gm{g}_us": round(statistics.median(v), 2) for g, v in times.items()},
               "bit_equal": all(torch.equal(base, o) for o in outs.values())}
        print(json.dumps(res), flush=True)
    os.environ.pop("DTFS_CROSS_GM", None)


if __name__ == "__main__":
    main()

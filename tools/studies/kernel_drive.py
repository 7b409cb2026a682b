"""Replay one model's serving-shape forward for kernel profiling.

    rocprofv3 --pmc SQ_WAVES ... --kernel-trace -d out -- python3 -m \\
        tools.studies.kernel_drive --model deepfm --rows 16384 --iters 20

Builds the bench preset of the model (random-init weights), captures the
forward at ``rows`` candidates (Zipf ids over 2^40, uniform weights) in a HIP
graph and replays it ``iters`` times: every kernel of a serving step at its
serving shape, nothing else (scripts/gpu_study.sh counters runs one counter pass per
invocation).
"""
from __future__ import annotations

import argparse

import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.models import build_model

PRESETS = {"deepfm": "deepfm_1gpu", "dcn_v2": "dcn_v2_fp8", "dcn": "reference_dcn", "wdl": "wdl_tiny_cpu",
           "dlrm": "dlrm_sharded8"}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="deepfm", choices=sorted(PRESETS))
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--table-rows", type=int, default=4_000_000,
                    help="dlrm: rows per table (30 tables; 4M = 15 GB, far past the 256 MiB Infinity Cache like "
                         "the served 60M-100M tables, but quick to initialise once per counter pass)")
    a = ap.parse_args(argv)
    cfg = load_preset(PRESETS[a.model]).model
    if a.model == "dlrm":
        cfg.table_rows = a.table_rows
    dev = torch.device("cuda:0")
    model = build_model(cfg, dev)
    ids, wts = SyntheticRequests(fields=cfg.num_fields, id_space=1 << 40, dist="zipf", seed=3).arrays(a.rows)
    ids, wts = torch.from_numpy(ids).to(dev), torch.from_numpy(wts).to(dev)
    out = torch.empty(a.rows, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            model(ids, wts, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model(ids, wts, out=out)
    for _ in range(a.iters):
        g.replay()
    torch.cuda.synchronize()
    print(f"kernel_drive: {a.model} x {a.rows} rows, {a.iters} replays, mean CTR {out.mean().item():.4f}", flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Flagship serving benchmark: DeepFM CTR fan-out over N MI355X GPUs.

Metric (BASELINE.json): CTR scores/sec for the whole node (+ request latency).
Config: DeepFM-style CTR, 1M x 64 bf16 embeddings, 43 fields, 3-layer MLP
(1024-512-256), client requests of 512 candidates (BASELINE config 2), fanned
out over N GPUs with RCCL all-to-all over xGMI (config 3 at N=4).

One timed step, on every rank, is a full serving round:

  1. ingest ``R`` serialized PredictRequests (512 candidates each; synthetic
     Zipf feature ids, uniform weights; TF ``tensor_content`` encoding). With
     ``--ingest arena`` (default) the native host code parses every request's
     protobuf framing in its pinned receive arena and writes descriptors; one
     SDMA copy moves the arena and a GPU kernel unpacks the candidate rows.
     With ``--ingest packed`` the host thread pool decodes rows itself;
  2. RCCL all-to-all of candidate rows over all GPUs -> model forward (gfx950
     kernels, one HIP graph) -> all-to-all of scores back -> D2H;
  3. encode R PredictResponses (``prediction_node`` float_val).

Four pipeline slots, three steps in flight: ingest of step k+3, the H2D of
k+1..k+2, the forward of k and the encode of k-1 overlap. Nothing is cached
across steps: every step re-parses and scores request bytes from a rotating
pool of distinct requests. Per-GPU work is fixed as N grows (weak scaling):
global batch = N * R * 512 candidates/step.

``--model`` picks the BASELINE config's preset: deepfm (configs 2/3), dlrm
(config 4: 100M-row tables sharded over the ranks), dcn_v2 (config 5: fp8
towers).

Launch: ``python bench.py`` (1 GPU) or, for N GPUs,
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
127.0.0.1 --master-port P bench.py --gpus N``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import json
import os
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from distributed_tf_serving_amd.config import ModelConfig, load_preset  # noqa: E402
from distributed_tf_serving_amd.parallel.embedding_sharding import (MI355X_HBM_BYTES,  # noqa: E402
                                                                    build_parallel_model)
from distributed_tf_serving_amd.ops import native  # noqa: E402
from distributed_tf_serving_amd.parallel.dist import init_from_env, shutdown  # noqa: E402
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine  # noqa: E402
from distributed_tf_serving_amd.serving.executor import ShardExecutor  # noqa: E402
from distributed_tf_serving_amd.serving.arena import ArenaLayout  # noqa: E402
from distributed_tf_serving_amd.serving.packing import PackedLayout  # noqa: E402
from distributed_tf_serving_amd.serving.pipeline import StepPipeline  # noqa: E402
from distributed_tf_serving_amd.client.synth import SyntheticRequests  # noqa: E402
from distributed_tf_serving_amd.utils.gc_tuning import tune_for_serving  # noqa: E402

BASELINE_VALUE = None  # the reference publishes no numbers
# --model -> configs/<preset>.yaml (BASELINE configs 2/3, 4, 5)
PRESETS = {"deepfm": "deepfm_1gpu", "dlrm": "dlrm_sharded8", "dcn_v2": "dcn_v2_fp8"}


def describe_model(cfg: ModelConfig) -> str:
    mlp = "-".join(str(d) for d in cfg.mlp_dims)
    if cfg.family == "dlrm":
        return (f"dlrm ({cfg.num_sparse} tables x {cfg.table_rows:,} rows x {cfg.embed_dim}, {cfg.num_dense} dense, "
                f"bottom {'-'.join(str(d) for d in cfg.bottom_mlp)}, top {mlp})")
    rows = f"{cfg.vocab_size // 1_000_000}M" if cfg.vocab_size % 1_000_000 == 0 else str(cfg.vocab_size)
    extra = f", {cfg.num_cross_layers} cross layers" if cfg.family in ("dcn", "dcn_v2") else ""
    return f"{cfg.family} ({rows}x{cfg.embed_dim} emb, {cfg.num_fields} fields, MLP {mlp}{extra})"


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="deepfm", choices=["deepfm", "dcn", "dcn_v2", "wdl", "dlrm"])
    ap.add_argument("--request-rows", type=int, default=512, help="candidates per client request (config batch)")
    ap.add_argument("--requests-per-gpu", type=int, default=32,
                    help="requests coalesced per GPU per step (32 x 512 = 16384 rows = the preset's max batch; "
                         "16 halves p50 latency for ~20%% less throughput)")
    ap.add_argument("--mode", default="alltoall", choices=["alltoall", "scatter", "local"])
    ap.add_argument("--encoding", default="raw", choices=["raw", "packed"],
                    help="raw = tensor_content; packed = int64_val/float_val like the reference client")
    ap.add_argument("--ingest", default="arena", choices=["arena", "packed"],
                    help="arena: host parses framing, GPU unpacks raw request bytes; packed: host decodes rows")
    ap.add_argument("--decode-threads", type=int, default=4,
                    help="native host pool per rank (4 measured best on a 16-CPU MI355X slice)")
    ap.add_argument("--pool", type=int, default=8, help="distinct pre-serialized steps per rank")
    ap.add_argument("--gemm-dtype", default=None, choices=["bf16", "fp8"],
                    help="default: the model preset's (fp8 towers for dcn_v2 = BASELINE config 5)")
    ap.add_argument("--table-rows", type=int, default=0, help="dlrm: rows per table (default: preset, 100M)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--slots", type=int, default=4, help="step slots per rank (steps in flight = slots - 1)")
    ap.add_argument("--loop", default="native", choices=["native", "python"],
                    help="native: per-step host loop in C++ (csrc/runtime/serving_loop.cpp); python: StepPipeline")
    ap.add_argument("--force-fanout", action="store_true",
                    help="keep the fan-out collectives on a 1-GPU run (exercises the N>1 step path)")
    ap.add_argument("--no-native-fanout", action="store_true",
                    help="N>1: issue collectives through torch.distributed instead of the C++ StepRunner")
    ap.add_argument("--json-extra", action="store_true", help="print extra diagnostics to stderr")
    ap.add_argument("--diag-skip-host", action="store_true",
                    help="DIAGNOSTIC ONLY (not a valid measurement): reuse decoded buffers to isolate GPU time")
    return ap.parse_args()


def main():
    a = parse_args()
    os.environ.setdefault("DTFS_HOST_THREADS", str(max(1, a.decode_threads)))
    ctx = init_from_env()
    world, rank = ctx.world, ctx.rank
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = ctx.device
    torch.manual_seed(1234)

    preset = PRESETS.get(a.model)
    cfg = load_preset(preset).model if preset else ModelConfig(family=a.model)
    if a.gemm_dtype:
        cfg.gemm_dtype = a.gemm_dtype
    if a.model == "dlrm":
        # config 4: 100M-row tables sharded over the ranks; a job too small to
        # hold them (e.g. 1 GPU: 384 GB > 288 GB) gets the largest row count
        # that fits its HBM budget, and reports it
        T, D = cfg.num_sparse, cfg.embed_dim
        rows = a.table_rows or cfg.table_rows
        fit = int(0.8 * MI355X_HBM_BYTES * world // (T * D * 2)) // 1_000_000 * 1_000_000
        if rows > fit:
            if rank == 0:
                print(f"note: {T} x {rows:,} rows do not fit {world} GPU(s); using {fit:,} rows/table",
                      file=sys.stderr)
            rows = fit
        cfg.table_rows = rows
    model = build_parallel_model(cfg, dev, ctx)
    F = cfg.num_fields
    layout = PackedLayout(F)
    B = a.requests_per_gpu * a.request_rows  # rows each GPU computes per step
    slots = a.slots
    ex = ShardExecutor(model, layout, [B], dev, use_graphs=not a.no_graphs, slots=slots)
    rows_in_max = B * (ctx.world if a.mode == "scatter" else 1)
    arena_layout = ArenaLayout(F, max_rows=max(1, rows_in_max))
    eng = FanoutEngine(ex, ctx, mode=a.mode, ingest=a.ingest, arena=arena_layout, force_fanout=a.force_fanout,
                       native_fanout=not a.no_native_fanout)
    eng.prepare(B)
    if eng.mode != "local":
        # one synthetic step checked against a local forward on every rank; a
        # failure anywhere switches every rank to the torch.distributed path
        eng.self_check(B, seed=rank)
    nat = native()

    rows_in = eng.contrib_rows(B)
    n_req = rows_in // a.request_rows
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=1000 + rank)
    pool = []
    for _ in range(max(1, a.pool)):
        pool.append([synth.serialized(a.request_rows, raw=(a.encoding == "raw")) for _ in range(n_req)])

    diag_pb = nat.parse_batch(pool[0], "feat_ids", "feat_wts", F) if pool[0] else None

    if a.ingest == "arena":
        # Requests are received into pinned arenas (a ring of a.pool receive
        # buffers, as an RDMA / shared-memory transport would deliver them);
        # every step re-parses its arena's framing on the host and the GPU
        # unpacks the raw payloads (csrc/kernels/ingest.hip).
        arenas, spans = [], []
        for reqs in pool:
            ar = arena_layout.alloc(pin=dev.type == "cuda")
            spans.append(arena_layout.place(ar, reqs) if reqs else [])
            arenas.append(ar)

    def decode(k: int, slot: int):
        reqs = pool[k % len(pool)]
        if not reqs:
            return None
        if a.ingest == "arena":
            ab = arena_layout.build(arenas[k % len(pool)], spans[k % len(pool)])
            errs = [e for e in ab.errors if e]
            if errs:
                raise RuntimeError(errs[0])
            return (ab, arenas[k % len(pool)])
        if a.diag_skip_host and k >= 2:  # diagnostic only: GPU pipeline without host decode
            return diag_pb
        pb = nat.parse_batch(reqs, "feat_ids", "feat_wts", F)
        buf = eng.host_in(B, slot)
        ids_v, wts_v = layout.ids(buf), layout.wts(buf)
        pb.decode(ids_v, wts_v)  # row chunks spread over the native host pool (DTFS_HOST_THREADS)
        errs = [e for e in pb.errors if e]
        if errs:
            raise RuntimeError(errs[0])
        return pb

    def encode(pb, scores: torch.Tensor):
        if pb is None:
            return []
        if isinstance(pb, tuple):
            pb = pb[0]
        return nat.encode_batch_responses("DCN", "serving_default", 1, "prediction_node", scores,
                                          list(pb.rows), list(pb.offsets))

    def launch(k: int, slot: int, ctx_k):
        if a.ingest == "arena" and ctx_k is not None:
            ab, ar = ctx_k
            return eng.launch(B, slot, src=ar, nbytes=ab.used_bytes)
        if a.ingest == "arena":  # a rank with no requests (scatter mode, rank > 0)
            return eng.launch(B, slot, nbytes=0)
        return eng.launch(B, slot)

    score_check = {"steps": 0, "mismatched_steps": 0}
    use_native_loop = a.loop == "native" and dev.type == "cuda" and a.ingest == "arena" and not a.no_graphs
    if use_native_loop:
        try:
            loop_slots = eng.loop_slots(B)
        except RuntimeError as e:  # e.g. a forward with collectives (sharded DLRM): Python pipeline
            if rank == 0:
                print(f"note: native loop unavailable ({e}); using the Python pipeline", file=sys.stderr)
            use_native_loop = False
    if use_native_loop:
        # the whole per-step host loop in C++ (csrc/runtime/serving_loop.cpp):
        # parse(k+3) || H2D(k+1..k+2) [SDMA] || step graph(k) [GPU] || encode(k-1)
        from distributed_tf_serving_amd.ops import hip

        nloop = hip().ServingLoop(eng.runner(), dict(depth=slots - 1, fields=F, max_rows=arena_layout.max_rows,
                                                     varint_chunks=arena_layout.varint_chunks,
                                                     version=1), loop_slots)
        for ar, sp in zip(arenas, spans):
            nloop.add_input(ar, sp)
        lat: list = []
        phase = {"parse": 0.0, "launch": 0.0, "gpu_wait": 0.0, "encode": 0.0}
        n_inputs = len(arenas)

        def run(n_steps: int, record: bool):
            st = nloop.run(n_steps, record)
            if st["errors"]:
                raise RuntimeError(f"{st['errors']} requests failed in the native loop")
            if record:
                # every replay of one input must give the same scores: a step
                # whose scores the host read before they landed shows up here
                ref = {}
                for k, v in enumerate(st["score_sum"]):
                    r = ref.setdefault(k % n_inputs, v)
                    if abs(v - r) > 1e-6 * max(1.0, abs(r)):
                        score_check["mismatched_steps"] += 1
                score_check["steps"] += len(st["score_sum"])
                lat.extend(x * 1e-6 for x in st["latency_us"])
                for k_src, k_dst in (("parse_us", "parse"), ("launch_us", "launch"), ("wait_us", "gpu_wait"),
                                     ("encode_us", "encode")):
                    phase[k_dst] += st[k_src] * 1e-6

        class _NoPipe:
            def reset_stats(self):
                lat.clear()
                for k in phase:
                    phase[k] = 0.0

            def close(self):
                pass

        pipe = _NoPipe()
    else:
        # decode(k+3) || H2D(k+1..k+2) [SDMA] || forward(k) [GPU] || encode(k-1)
        pipe = StepPipeline(eng, B, slots=slots, depth=slots - 1, produce=decode,
                            consume=lambda k, pb, scores: encode(pb, scores), launch=launch)
        phase = pipe.phase
        lat = pipe.latencies

        def run(n_steps: int, record: bool):
            pipe.run(n_steps, record=record)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if ctx.is_distributed:
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    tune_for_serving()  # same process tuning as the gRPC server (utils/gc_tuning.py)
    run(max(1, a.warmup), record=False)
    sync()
    pipe.reset_stats()
    t0 = time.perf_counter()
    run(a.steps, record=True)
    sync()
    el = time.perf_counter() - t0

    t = torch.tensor([el], dtype=torch.float64, device=dev if ctx.backend == "nccl" else "cpu")
    if ctx.is_distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max = float(t.item())
    total_scores = world * B * a.steps
    value = total_scores / el_max
    p50 = statistics.median(lat) * 1e3 if lat else None
    p99 = float(np.percentile(lat, 99)) * 1e3 if lat else None
    if rank == 0:
        out = {
            "metric": "CTR scores/sec (whole node)",
            "value": round(value, 1),
            "unit": "scores/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(value / BASELINE_VALUE, 4),
            "dtype": cfg.gemm_dtype,
            "data": "synthetic (zipf feature ids over 2^40, uniform weights; random-init weights)",
            "config": {
                "model": describe_model(cfg),
                "global_batch": world * B,
                "request_rows": a.request_rows,
                "requests_per_gpu_per_step": a.requests_per_gpu,
                "seq_len": None,
                "parallelism": f"candidate-dp{world} ({eng.mode} fan-out over RCCL"
                               + (", native C++ step" if eng.native_fanout_active else "") + ")" + (
                    f" + embedding-mp{world} ({len(model.plan.row_wise())} row-wise tables, all-to-all)"
                    if hasattr(model, "plan") else ""),
                "encoding": a.encoding,
            },
            "p50_request_ms": None if p50 is None else round(p50, 3),
            "p99_request_ms": None if p99 is None else round(p99, 3),
        }
        if score_check["steps"]:
            out["score_check"] = ("ok" if not score_check["mismatched_steps"] else
                                  f"{score_check['mismatched_steps']}/{score_check['steps']} steps differ")
        print(json.dumps(out), flush=True)
        if a.json_extra:
            per = {k: round(v / a.steps * 1e6, 1) for k, v in phase.items()}
            print(json.dumps({"host_phase_us_per_step": per}), file=sys.stderr, flush=True)
    pipe.close()
    shutdown()


if __name__ == "__main__":
    main()

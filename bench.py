#!/usr/bin/env python
"""Flagship serving benchmark: DeepFM CTR served by the native live server on N MI355X GPUs.

Metric (BASELINE.json): CTR scores/sec for the whole node + p50 request latency
at a fixed QPS. Config: DeepFM-style CTR, 1M x 64 bf16 embeddings, 43 fields,
3-layer MLP (1024-512-256), client requests of 512 candidates (BASELINE config
2); at N > 1 every request's candidates are fanned out over all GPUs with RCCL
all-to-all over xGMI (config 3 at N=4).

What is timed is the SERVED path, the one the gRPC front door and in-process
clients use (serving/live.py -> csrc/runtime/live_server.cpp):

  client threads (native load generator, csrc/runtime/loadgen.cpp) submit
  serialized PredictRequests (synthetic Zipf ids, uniform weights, TF
  ``tensor_content``) -> validation + admission into the open dynamic batch ->
  ONE copy of the request bytes into a pinned arena -> launcher thread: batch
  closed at max rows (32 x 512 = 16384) / timeout, framing parse, SDMA H2D,
  step kernels (GPU unpack + gather + FM + MFMA GEMMs + fused head; at N > 1 the
  native fan-out step with its two all-to-alls) -> completer thread: bounded
  wait, one PredictResponse encoded per request -> the client's completion.

One "step" = one GPU batch = ``--requests-per-gpu`` requests on every rank.
The closed loop keeps ``(slots + 2) x R`` requests outstanding; the clock runs
from the completion that ends warmup step W to the one that ends step W + K,
inside one continuous run (the pipeline stays primed across the boundary).
N=1 also reports: scores checked against an fp32 CPU forward of the same
weights, the p50/p99 of an open-loop run at ``--qps`` (fixed offered load), and
the literal config-2 point (one 512-candidate request per step, concurrency 1).

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

from distributed_tf_serving_amd.config import ModelConfig, ServingConfig, load_preset  # noqa: E402
from distributed_tf_serving_amd.parallel.embedding_sharding import (MI355X_HBM_BYTES,  # noqa: E402
                                                                    build_parallel_model)
from distributed_tf_serving_amd.ops import native  # noqa: E402
from distributed_tf_serving_amd.parallel.dist import init_from_env, shutdown  # noqa: E402
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine  # noqa: E402
from distributed_tf_serving_amd.serving.executor import ShardExecutor  # noqa: E402
from distributed_tf_serving_amd.serving.arena import ArenaLayout  # noqa: E402
from distributed_tf_serving_amd.serving.live import LiveScheduler  # noqa: E402
from distributed_tf_serving_amd.serving.packing import PackedLayout, layout_for  # noqa: E402
from distributed_tf_serving_amd.client.synth import SyntheticRequests  # noqa: E402
from distributed_tf_serving_amd.utils.gc_tuning import tune_for_serving  # noqa: E402

BASELINE_VALUE = None  # the reference publishes no numbers
# --model -> configs/<preset>.yaml (BASELINE configs 2/3, 4, 5)
PRESETS = {"deepfm": "deepfm_1gpu", "dlrm": "dlrm_sharded8", "dcn_v2": "dcn_v2_fp8"}


def dtype_label(cfg: ModelConfig) -> str:
    """Compute dtype of the step. fp8 models keep the small MLP tail in bf16
    (models/ctr.py DCNv2: the cross layers + the first MLP layer, 97 % of the
    FLOPs, run MX-fp8; fp32 accumulation everywhere)."""
    if cfg.gemm_dtype == "fp8":
        return "fp8 (e4m3 cross layers + first MLP layer, 97 % of FLOPs) + bf16 MLP tail"
    return cfg.gemm_dtype


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
    ap.add_argument("--prime-steps", type=int, default=1000,
                    help="server start-up load: untimed steps of the same continuous closed loop run BEFORE the "
                         "--warmup steps (clocks, caches and host threads reach steady state, as in a server that "
                         "has been up for a while); the timed window is still exactly --steps steps")
    ap.add_argument("--model", default="deepfm", choices=["deepfm", "dcn", "dcn_v2", "wdl", "dlrm"])
    ap.add_argument("--request-rows", type=int, default=512, help="candidates per client request (config batch)")
    ap.add_argument("--requests-per-gpu", type=int, default=32,
                    help="requests per GPU batch (32 x 512 = 16384 rows = the preset's max batch)")
    ap.add_argument("--peer-comm", type=int, default=None,
                    help="one-shot peer exchange (csrc/kernels/peer.hip) for fan-out / step-program messages of at "
                         "most this many bytes per peer (1 = 64 KiB, 0 = RCCL only; default: $DTFS_PEER_COMM or 0)")
    ap.add_argument("--scatter-path", default="shared", choices=["shared", "rccl"],
                    help="scatter mode: shared = each GPU DMAs its share of rank 0's shared request arenas; "
                         "rccl = RCCL scatter / gather of packed rows")
    ap.add_argument("--mode", default=None, choices=["alltoall", "scatter", "local"],
                    help="N > 1: alltoall = every request fanned out over all GPUs (config 3, default); local = "
                         "one independent replica per GPU (default for dlrm: its tables are sharded instead and "
                         "every step exchanges embeddings); scatter = rank 0 is the only front door")
    ap.add_argument("--feature-weights", default="uniform", choices=["uniform", "ones"],
                    help="request feature weights: uniform in (0, 1] (default) or all 1.0 as the reference client "
                         "sends them (DCNClient.java:67-73; host narrowing then ships no weight bytes)")
    ap.add_argument("--encoding", default="raw", choices=["raw", "packed"],
                    help="raw = tensor_content; packed = int64_val/float_val like the reference client")
    ap.add_argument("--decode-threads", type=int, default=4,
                    help="native host pool per rank (4 measured best on a 16-CPU MI355X slice)")
    ap.add_argument("--client-threads", type=int, default=8, help="load-generator submitting threads per rank")
    ap.add_argument("--open-loop-threads", type=int, default=8,
                    help="submitting threads per rank of the open-loop runs (fixed QPS, latency sweep). Each "
                         "512-candidate request costs its submitter ~25 us of copying and narrowing (~6.5 CPUs of "
                         "work at 90 %% of a ~290 k requests/s capacity, whatever the thread count); 12 threads "
                         "measured no better and, on a box whose 16-CPU quota was contended, worse")
    ap.add_argument("--pool", type=int, default=64, help="distinct pre-serialized requests per rank")
    ap.add_argument("--gemm-dtype", default=None, choices=["bf16", "fp8"],
                    help="default: the model preset's (fp8 towers for dcn_v2 = BASELINE config 5)")
    ap.add_argument("--table-rows", type=int, default=0, help="dlrm: rows per table (default: preset, 100M)")
    ap.add_argument("--shard-tables", action="store_true",
                    help="dlrm: shard the tables even on one GPU (exercises the embedding-exchange step program)")
    ap.add_argument("--exchange", default=None, choices=["alltoall", "peer"],
                    help="dlrm sharded tables: ids + rows through RCCL all-to-alls, or rows loaded from the owner's "
                         "HBM over xGMI behind a per-rank hot-row replica cache (default: the preset's)")
    ap.add_argument("--hot-cache-rows", type=int, default=None,
                    help="peer exchange: replica cache rows per rank (default: the config's; 0 = no cache)")
    ap.add_argument("--cache-learn-rounds", type=int, default=2,
                    help="peer exchange: untimed learning rounds before the clock, each a pass over the request "
                         "pool with every candidate's remote keys sampled, then a cache refresh (a server "
                         "refreshes every second)")
    ap.add_argument("--cache-learn-requests", type=int, default=0,
                    help="peer exchange: requests per learning round (0: the whole request pool)")
    ap.add_argument("--cache-refresh-s", type=float, default=0.0,
                    help="peer exchange: > 0 keeps the background refresher running (this period) through the "
                         "timed run, so the clock covers the refreshes' cost")
    ap.add_argument("--stream-pool", type=int, default=4096,
                    help="peer exchange: distinct pre-serialized requests per rank (a long, non-repeating stream "
                         "for the replica cache to learn; --pool for every other model)")
    ap.add_argument("--small-buckets", default=None,
                    help="extra padding buckets (rows per GPU) below the full step, so a lightly loaded server "
                         "runs a step sized to what is queued (TF-Serving allowed_batch_sizes; at N > 1 every "
                         "rank agrees on the largest bucket any rank needs); '' = only the full step. 2048: "
                         "bench/bucket_cost.py on MI355X - a 512- or 1024-row step costs 64-66 us pipelined "
                         "(launch-chain bound), a 2048-row one 79 us, so smaller buckets only saturate at 20k QPS "
                         "of 512-row requests. Default 2048; dcn_v2 (a 0.6 ms full step) 2048,4096,8192")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--slots", type=int, default=4, help="step slots per rank (steps in flight)")
    ap.add_argument("--batch-timeout-us", type=int, default=200)
    ap.add_argument("--qps", type=float, default=20000.0,
                    help="offered load of the fixed-QPS latency run, whole node (requests/s; 0 = skip); at N > 1 "
                         "split evenly over the front-door ranks")
    ap.add_argument("--qps-seconds", type=float, default=1.0)
    ap.add_argument("--qps-sweep", default="0.25,0.5,0.75,0.9",
                    help="latency vs offered load: open-loop runs at these fractions of the measured capacity "
                         "(requests/s of the throughput run), p50 / p99 each ('' = off)")
    ap.add_argument("--force-fanout", action="store_true",
                    help="keep the fan-out collectives on a 1-GPU run (exercises the N>1 step path)")
    ap.add_argument("--step-timeout-s", type=float, default=30.0,
                    help="a step not finished by then fails the run instead of hanging it")
    ap.add_argument("--h2d-wait", default=None, choices=["host", "device", "feed"],
                    help="local steps: the launcher waits for each step's H2D copy on the host before it enqueues "
                         "the kernels (host: copies never overlap), the compute stream waits on the copy's event on "
                         "the device (device), or a feeder thread enqueues the kernels once the host sees the copy "
                         "landed while the launcher issues the next copies (feed); default: the runtime's (feed)")
    ap.add_argument("--embed-geometry", default=None, metavar="WAVES,ROWS",
                    help="pipelined gather geometry for a study: resident-wave cap and rows in flight per wave "
                         "(default: the kernel's 4096,1)")
    ap.add_argument("--no-narrow", action="store_true",
                    help="ship raw int64 ids / fp32 weights to the GPU instead of host-narrowed 3-byte / int32 rows "
                         "with fp32 weights")
    ap.add_argument("--json-extra", action="store_true", help="print extra diagnostics to stderr")
    ap.add_argument("--reference-workload", action="store_true",
                    help="the reference's own run instead (DCNClient.java:25-42, 57-74, 205-241): model DCN, requests "
                         "of 1500 candidates with ids 1..43 and weights 1.0 encoded like the reference client "
                         "(int64_val / float_val), 6 closed-loop clients x --ref-requests requests; prints the "
                         "reference's output lines and a JSON summary. At N > 1 rank 0 is the only front door and "
                         "every request is scattered over the GPUs (the reference's 3-host fan-out, inside a node)")
    ap.add_argument("--ref-requests", type=int, default=1000, help="requests per client thread (reference: 1000)")
    ap.add_argument("--ref-clients", type=int, default=6, help="closed-loop client threads (reference: 6)")
    ap.add_argument("--over-grpc", action="store_true",
                    help="--reference-workload on 1 GPU: the clients are a separate process of native h2c gRPC "
                         "clients (client/native_load.py) talking to the native gRPC front door "
                         "(serving/native_front.py) over TCP, instead of in-process submits")
    ap.add_argument("--grpc-threads", type=int, default=4, help="--over-grpc: front-door event-loop threads")
    ap.add_argument("--print-requests", action="store_true",
                    help="--reference-workload: also print one 'Time cost' line per request, like the reference")
    a = ap.parse_args()
    if a.reference_workload:
        a.model, a.request_rows, a.encoding = "dcn", 1500, "packed"
        if a.mode is None:
            a.mode = "scatter"
    return a


def build(a, ctx):
    """Model, executor and fan-out engine of this rank (arena ingest)."""
    world, rank = ctx.world, ctx.rank
    dev = ctx.device
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
        if a.exchange:
            cfg.embedding_exchange = a.exchange
        if a.hot_cache_rows is not None:
            cfg.hot_cache_rows = a.hot_cache_rows
    # CPU (gloo): the step's collectives run on the live server's launcher
    # thread, so they get a group of their own (the main thread syncs phases
    # on the default group)
    step_group = dist.new_group(backend="gloo") if (world > 1 and dev.type != "cuda") else None
    if a.embed_geometry and dev.type == "cuda":  # before any capture: the graphs bake the grid in
        from distributed_tf_serving_amd.ops import hip

        w, r = (int(x) for x in a.embed_geometry.split(","))
        hip().set_embed_wave_cap(w, r)
    model = build_parallel_model(cfg, dev, ctx, shard_tables="on" if a.shard_tables else "auto", group=step_group)
    F = cfg.num_fields
    B = a.requests_per_gpu * a.request_rows  # rows each GPU computes per step
    if a.reference_workload:
        # rows per GPU when k of the clients' 1500-candidate requests share a step
        # (scatter at N > 1: rank 0's batch of k x 1500 rows is split over N GPUs)
        split = world if (a.mode or "scatter") == "scatter" and world > 1 else 1
        per = [-(-(k * a.request_rows) // (split * 64)) * 64 for k in range(1, a.ref_clients + 1)]
        B = per[-1]
        a.small_buckets = ",".join(str(b) for b in sorted(set(per[:-1])))
    sharded = getattr(model, "has_collectives", False) or (a.model == "dlrm" and a.shard_tables)
    if a.mode is None:
        a.mode = "local" if a.model == "dlrm" else "alltoall"
    if sharded and a.mode != "local":
        raise SystemExit("dlrm with sharded tables runs --mode local (the embedding exchange is the fan-out)")
    mode = a.mode if world > 1 else ("alltoall" if a.force_fanout else "local")
    if a.small_buckets is None:
        # a full DCN-v2 step is 0.6 ms: intermediate buckets keep a lightly
        # loaded server from padding every step to the full one
        a.small_buckets = "2048,4096,8192" if cfg.family == "dcn_v2" else "2048"
    small = [int(x) for x in a.small_buckets.split(",") if x.strip()] if a.small_buckets else []
    # an all-to-all splits every rank's rows evenly over the GPUs
    small = [b for b in small if mode != "alltoall" or b % world == 0]
    buckets = sorted({b for b in small if 0 < b < B} | {B})
    # scatter on one node: every rank DMAs its share of rank 0's shared arenas
    # (csrc/runtime/shared_scatter.h); --scatter-path rccl: the RCCL scatter
    shared = mode == "scatter" and world > 1 and a.scatter_path == "shared"
    # fan-out rows travel narrow (int32 table rows + fp32 weights: 8 instead of 12 bytes per feature over xGMI)
    layout = (layout_for(cfg, not a.no_narrow) if mode != "local" and not shared else PackedLayout(F))
    ex = ShardExecutor(model, layout, buckets, dev, use_graphs=not a.no_graphs, slots=a.slots)
    rows_in_max = B * (world if mode == "scatter" else 1)
    arena_layout = ArenaLayout(F, max_rows=max(1, rows_in_max), gpu_varint=not shared)
    seg = None
    if shared:
        from distributed_tf_serving_amd.parallel.shared_scatter import live_narrowing, scatter_for_engine

        nm, nw = live_narrowing(model, dev.type == "cuda")
        seg = scatter_for_engine(ctx, F, arena_layout.capacity, a.slots, B, tag="bench", narrow_modulo=nm,
                                 narrow_wts_cols=nw)
    eng = FanoutEngine(ex, ctx, mode=mode, ingest="arena", arena=arena_layout, force_fanout=a.force_fanout,
                       group=step_group, shared_scatter=seg)
    for b in buckets:
        eng.prepare(b)
    if a.h2d_wait and dev.type == "cuda":
        eng.runner().host_wait_h2d = a.h2d_wait == "host"
        eng.runner().feed_h2d = a.h2d_wait == "feed"
    if eng.program_active or eng.mode != "local":
        # one synthetic step of every bucket checked against a local / eager
        # forward on every rank (collective): a fan-out that scores wrong is
        # a failed run, not a silent fallback
        for b in buckets:
            if not eng.self_check(b, seed=rank):
                raise SystemExit(f"rank {rank}: the fan-out step's scores differ from a local forward (bucket {b})")
        if dev.type == "cuda" and eng.mode != "local" and eng.scatter is None and not eng.native_fanout_active:
            raise SystemExit(f"rank {rank}: the native fan-out step is not active")
    return cfg, model, eng, B


def request_pool(a, ctx, eng, B, F):
    rows_in = eng.contrib_rows(B)
    n_req = rows_in // a.request_rows
    if a.reference_workload:  # every candidate ids 1..43, weights 1.0 (DCNClient.java:57-74)
        synth = SyntheticRequests(fields=F, dist="reference")
        return ([synth.serialized(a.request_rows, raw=False)] if rows_in else []), n_req
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=1000 + ctx.rank,
                              weights=a.feature_weights)
    peer = getattr(getattr(getattr(eng.ex, "model", None), "emb", None), "peer", None) is not None
    n = max(1, a.stream_pool if peer else a.pool) if n_req else 0
    return [synth.serialized(a.request_rows, raw=(a.encoding == "raw")) for _ in range(n)], n_req


def fresh_hit_rate(cfg, model, ctx, rows: int = 32768) -> float:
    """Fraction of remote lookups of a FRESH draw of the synthetic stream
    (another seed than the served pool) that the installed hot set holds."""
    import numpy as np

    from distributed_tf_serving_amd.parallel.hot_cache import KEY_SHIFT

    cache, peer = model.cache, model.emb.peer
    ids, _ = SyntheticRequests(fields=cfg.num_fields, id_space=1 << 40, dist="zipf",
                               seed=99991 + ctx.rank).arrays(rows)
    hot, col0 = int(getattr(model, "hot", 1)), cfg.num_dense
    keys = cache.keys.cpu().numpy()
    hit = tot = 0
    for t in range(peer.T):
        if not bool(peer.tremote_cpu[t]):
            continue
        v = ids[:, col0 + t * hot:col0 + (t + 1) * hot].astype(np.int64) % np.int64(peer.rows[t])
        k = (np.int64(t) << KEY_SHIFT) | v.reshape(-1)
        pos = np.clip(np.searchsorted(keys, k), 0, max(0, keys.size - 1))
        hit += int((keys[pos] == k).sum()) if keys.size else 0
        tot += k.size
    return round(hit / tot, 4) if tot else 0.0


def cache_oracle(a, cfg, model, ctx, n_pool: int, extra_k=()) -> dict:
    """Hit rate of the EXACT top-k remote keys of the served request pool (the
    same generator and seed as request_pool; every request equally likely): an
    upper bound for any hot set of k rows on this stream, at k = 1 M / 8 M /
    64 M and the cache's capacity / installed rows (extra_k)."""
    import numpy as np

    from distributed_tf_serving_amd.parallel.hot_cache import KEY_SHIFT

    peer = model.emb.peer
    hot, col0 = int(getattr(model, "hot", 1)), cfg.num_dense
    synth = SyntheticRequests(fields=cfg.num_fields, id_space=1 << 40, dist="zipf", seed=1000 + ctx.rank,
                              weights=a.feature_weights)
    remote = [t for t in range(peer.T) if bool(peer.tremote_cpu[t])]
    keys = []
    for _ in range(n_pool):
        ids, _ = synth.arrays(a.request_rows)
        for t in remote:
            v = ids[:, col0 + t * hot:col0 + (t + 1) * hot].astype(np.int64) % np.int64(peer.rows[t])
            keys.append((np.int64(t) << KEY_SHIFT) | v.reshape(-1))
    if not keys:
        return {}
    _, counts = np.unique(np.concatenate(keys), return_counts=True)
    counts = np.sort(counts)[::-1]
    csum, total = np.cumsum(counts), float(counts.sum())
    ks = sorted({1 << 20, 8 << 20, 64 << 20, *[int(k) for k in extra_k if k > 0]})
    return {"distinct_keys": int(counts.size), "lookups": int(total),
            "hit_rate_at": {str(k): round(float(csum[min(k, counts.size) - 1]) / total, 4) for k in ks}}


def fp32_check(cfg, model, live, request: bytes) -> dict:
    """Scores of one served request vs an fp32 forward of the same weights on
    the CPU (the ops' reference math)."""
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    if cfg.family == "dlrm" and model.param_bytes() > (4 << 30):
        return fp32_check_dlrm_sparse(cfg, model, live, request)
    if model.param_bytes() > (4 << 30):
        return {"status": "skipped (model too large for a CPU copy)"}
    ref = build_model(cfg, "cpu")
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    if cfg.gemm_dtype == "fp8":
        for m in ref.modules():
            if hasattr(m, "quantize_fp8") and getattr(m, "fp8", False):
                m.quantize_fp8()
    req = pb.PredictRequest.FromString(request)
    ids = torch.from_numpy(T.to_ndarray(req.inputs["feat_ids"]))
    wts = torch.from_numpy(T.to_ndarray(req.inputs["feat_wts"]))
    want = ref(ids, wts).float()
    resp = pb.PredictResponse.FromString(live.predict_bytes(request, 30.0))
    got = torch.from_numpy(T.to_ndarray(resp.outputs["prediction_node"]))
    diff = float((got - want).abs().max())
    tol = 5e-2 if cfg.gemm_dtype == "fp8" else 2e-2
    return {"status": "ok" if diff <= tol else "MISMATCH", "max_abs_diff": round(diff, 6), "tol": tol,
            "rows": int(got.numel())}


def fp32_check_dlrm_sparse(cfg, model, live, request: bytes) -> dict:
    """DLRM tables too large for a CPU copy (30 x 60M-100M rows): the fp32
    reference rebuilds ONLY the table rows the request references, from the
    tables' hashed init (models/layers.py hashed_rows_at: a value depends only
    on (seed, table, row), so it is the GPU table's content, rounded to its
    bf16), copies the dense towers, and runs the CPU reference math."""
    from distributed_tf_serving_amd.models.ctr import DLRM
    from distributed_tf_serving_amd.models.layers import hashed_rows_at
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    dense = getattr(model, "dense", model)  # ShardedDLRM keeps its towers in .dense
    ref = DLRM(cfg, "cpu", materialize_tables=False).eval()
    sd = {k: v.detach().cpu() for k, v in dense.state_dict().items() if not k.startswith("emb")}
    ref.load_state_dict(sd, strict=False)
    req = pb.PredictRequest.FromString(request)
    ids = torch.from_numpy(T.to_ndarray(req.inputs["feat_ids"])).long()
    wts = torch.from_numpy(T.to_ndarray(req.inputs["feat_wts"])).float()
    nd, Tn, hot, D = cfg.num_dense, cfg.num_sparse, max(1, int(cfg.multi_hot)), cfg.embed_dim
    B = ids.shape[0]
    rows = torch.remainder(ids[:, nd:], cfg.table_rows).view(B, Tn, hot)
    emb = torch.empty(B, Tn, hot, D)
    for t in range(Tn):
        v = hashed_rows_at(rows[:, t].reshape(-1), D, t, cfg.seed, ref.table_bound)
        emb[:, t] = v.to(torch.bfloat16).float().view(B, hot, D)  # the table stores bf16
    if hot == 1:
        e = emb[:, :, 0].to(torch.bfloat16)
    else:  # weighted bags, pooled in fp32 and stored bf16 (the K1b kernel's output)
        e = (emb * wts[:, nd:].view(B, Tn, hot, 1)).sum(2).to(torch.bfloat16)
    with torch.no_grad():
        want = ref.interact_and_top(ref.bottom_out(wts), e).float()
    resp = pb.PredictResponse.FromString(live.predict_bytes(request, 30.0))
    got = torch.from_numpy(T.to_ndarray(resp.outputs["prediction_node"]))
    diff = float((got - want).abs().max())
    tol = 2e-2
    return {"status": "ok" if diff <= tol else "MISMATCH", "max_abs_diff": round(diff, 6), "tol": tol,
            "rows": int(got.numel()), "reference": f"sparse: {B * Tn * hot} referenced table rows rebuilt on the CPU"}


STAGES = ("sched_lag", "admit", "batch", "step", "encode", "deliver")  # csrc/runtime/loadgen.h Stages


def stage_breakdown(r: dict):
    """Where the requests of a load run spent their latency (this rank's front
    door): each stage's p50 / p99, and its mean over the requests at or above
    the run's p99 latency - the tail's own breakdown."""
    lat = np.asarray(r.get("latency_us", []), dtype=np.float64)
    st = np.asarray(r.get("stages_us", np.zeros((0, len(STAGES)))), dtype=np.float64)
    if lat.size == 0 or st.shape != (lat.size, len(STAGES)):
        return None
    tail = st[lat >= np.percentile(lat, 99)]
    r1 = lambda v: round(float(v), 1)  # noqa: E731
    return {"p50_us": {k: r1(np.percentile(st[:, i], 50)) for i, k in enumerate(STAGES)},
            "p99_us": {k: r1(np.percentile(st[:, i], 99)) for i, k in enumerate(STAGES)},
            "tail_mean_us": {k: r1(tail[:, i].mean()) for i, k in enumerate(STAGES)} if len(tail) else None,
            "tail_requests": int(len(tail))}


def host_sched_counters() -> dict:
    """Host-side scheduling counters of this process (what a latency tail
    caused by the host looks like): the cgroup's CPU quota and throttling
    (cgroup v2 cpu.max / cpu.stat), the process's CPU time and its voluntary /
    involuntary context switches (getrusage). Diff two readings."""
    import resource

    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
        out["cpu_quota_cpus"] = None if q == "max" else round(int(q) / int(per), 2)
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for ln in f:
                k, v = ln.split()
                if k in ("nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
    except (OSError, ValueError):
        pass
    ru = resource.getrusage(resource.RUSAGE_SELF)
    out.update(cpu_s=ru.ru_utime + ru.ru_stime, nvcsw=ru.ru_nvcsw, nivcsw=ru.ru_nivcsw, wall_s=time.monotonic())
    return out


def host_sched_delta(a: dict, b: dict) -> dict:
    d = {k: b[k] - a[k] for k in b if k in a and k != "cpu_quota_cpus" and b[k] is not None and a[k] is not None}
    wall = d.pop("wall_s", 0.0)
    d["cpus_busy"] = round(d.pop("cpu_s", 0.0) / wall, 2) if wall > 0 else None
    d["wall_s"] = round(wall, 2)
    d["cpu_quota_cpus"] = b.get("cpu_quota_cpus")
    return d


def pct(lat_us, q):
    return round(float(np.percentile(lat_us, q)) * 1e-3, 3) if len(lat_us) else None


def run_live(a, ctx, cfg, model, eng, B):
    world, rank, dev = ctx.world, ctx.rank, ctx.device
    F = cfg.num_fields
    pool, n_req = request_pool(a, ctx, eng, B, F)
    conc = (a.slots + 2) * max(1, n_req)
    untimed = a.prime_steps + a.warmup  # one continuous run: prime, then warmup, then the K timed steps
    buckets = list(eng.ex.buckets)
    sc = ServingConfig(max_batch_rows=B, allowed_batch_sizes=tuple(buckets), batch_timeout_us=a.batch_timeout_us,
                       max_queued_rows=1 << 24, max_request_rows=1 << 20)
    # steps with collectives are agreed with the other ranks through the
    # shared-memory step control: launched only when some rank has requests,
    # at the smallest bucket that holds every rank's batch
    control = None
    if eng.lockstep and world > 1:
        from distributed_tf_serving_amd.ops import hip
        from distributed_tf_serving_amd.parallel.control import control_for_job

        control = control_for_job(hip() if dev.type == "cuda" else native(), ctx, "bench")
    live = LiveScheduler(eng, sc, buckets=buckets, depth=a.slots, control=control, step_timeout_s=a.step_timeout_s,
                         start_paused=control is not None, narrow=not a.no_narrow, peer_timeout_s=a.step_timeout_s)
    extra = {}
    if eng.self_checks:  # every bucket's fan-out step vs a local forward of the same rows, at start-up
        extra["self_check"] = {"atol": 1e-5, "buckets": eng.self_checks}
    if world == 1 and pool:
        extra["fp32_check"] = fp32_check(cfg, model, live, pool[0])
    # phase barriers of the main thread: a CPU group of their own (the step's
    # collectives, if any, run on the launcher thread on other communicators)
    phase = dist.new_group(backend="gloo") if ctx.is_distributed else None

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if ctx.is_distributed:
            dist.barrier(group=phase)

    tune_for_serving()  # same process tuning as the gRPC server (utils/gc_tuning.py)
    sync()
    if control is not None:
        live.resume()  # every rank is past its start-up collectives: steps may begin
    timeout_us = int(a.step_timeout_s * 1e6)
    cache = getattr(model, "cache", None)
    if cache is not None and pool:
        # peer exchange: serve the request pool with every candidate's remote
        # keys sampled (the kernels read the period from the cache descriptor,
        # the captured graphs stay), installing the hot set after each pass;
        # then back to sampling every sample_every-th candidate (the refresher
        # is off while the clock runs: a synthetic stream's hot set does not drift)
        cache.set_sample_period(1)
        per_pass = a.cache_learn_requests if a.cache_learn_requests > 0 else max(max(8, a.warmup) * n_req, len(pool))
        # at most half the ring's keys per refresh: pushes land in 64 segments
        # by block, and a segment that wraps overwrites keys not yet counted
        keys_per_req = a.request_rows * max(1, model.emb.peer.remote_tables) * int(getattr(model, "hot", 1))
        chunk = max(n_req, min(per_pass, cache.ring.numel() // max(1, 2 * keys_per_req)))
        for _ in range(a.cache_learn_rounds):
            done = 0
            while done < per_pass:
                n = min(chunk, per_pass - done)
                # this chunk's slice of the pool (run_load starts at its list's
                # first request: the whole pool each time would replay the same
                # first n requests every chunk and learn only their keys)
                part = [pool[(done + i) % len(pool)] for i in range(n)]
                live.run_load(part, warmup=0, count=n, concurrency=conc, threads=a.client_threads,
                              timeout_us=timeout_us)
                cache.refresh()
                done += n
        cache.set_sample_period(0)
        sync()
        cache.reset_counts()
        if a.cache_refresh_s > 0:  # the serving configuration: refreshes run while the clock does
            cache.start(a.cache_refresh_s)
    steps0 = live.stats()["steps"]
    if pool:
        r = live.run_load(pool, warmup=untimed * n_req, count=a.steps * n_req, concurrency=conc,
                          threads=a.client_threads, timeout_us=timeout_us)
    else:  # a rank without requests (scatter followers): its live server joins rank 0's steps
        r = {"window_us": 0.0, "latency_us": [], "errors": 0, "ok": 0}
    st_load = live.stats()
    cache_counts = cache.counts() if cache is not None else None  # the throughput run's lookups
    window_s = r["window_us"] * 1e-6
    if r["errors"]:
        print(f"rank {rank}: {r['errors']} requests failed: {r.get('first_error')}", file=sys.stderr, flush=True)
    lat = r["latency_us"]
    extra["p50_request_ms"], extra["p99_request_ms"] = pct(lat, 50), pct(lat, 99)
    extra["requests_failed"] = int(r["errors"])

    # fixed offered load (whole node), split over the front-door ranks
    fronts = world if eng.contrib_rows(B) and eng.mode != "scatter" else 1
    if a.qps > 0:
        sync()
        q = {"latency_us": [], "errors": 0}
        if pool:
            n = max(200, int(a.qps / fronts * a.qps_seconds))
            q = live.run_load(pool, warmup=n // 10, count=n, qps=a.qps / fronts, threads=a.open_loop_threads,
                              timeout_us=timeout_us)
        p50, p99 = pct(q["latency_us"], 50), pct(q["latency_us"], 99)
        red = torch.tensor([p50 or 0.0, p99 or 0.0, float(q["errors"])], dtype=torch.float64)
        if ctx.is_distributed:  # the slowest front door's percentiles
            dist.all_reduce(red, op=dist.ReduceOp.MAX, group=phase)
        extra["fixed_qps"] = {"qps": a.qps, "front_doors": fronts, "request_rows": a.request_rows,
                              "scores_per_s": round(a.qps * a.request_rows, 1),
                              "p50_ms": round(float(red[0]), 3), "p99_ms": round(float(red[1]), 3),
                              "errors": int(red[2]), "stages": stage_breakdown(q)}
        extra["p50_at_fixed_qps_ms"] = extra["fixed_qps"]["p50_ms"]
    fracs = [float(x) for x in a.qps_sweep.split(",") if x.strip()] if a.qps_sweep else []
    hs0 = host_sched_counters()
    if fracs:  # every rank takes part (the collectives below); ranks without requests only follow
        # the throughput run's request rate, whole node (slowest rank's window)
        w = torch.tensor([window_s], dtype=torch.float64)
        if ctx.is_distributed:
            dist.all_reduce(w, op=dist.ReduceOp.MAX, group=phase)
        cap_qps = a.steps * n_req / float(w[0]) * fronts if float(w[0]) > 0 else 0.0
        sweep = []
        for f in fracs:
            qps = f * cap_qps
            sync()
            q = {"latency_us": [], "errors": 0, "window_us": 0.0}
            n = max(200, int(qps / fronts * a.qps_seconds))
            if pool and qps > 0:
                q = live.run_load(pool, warmup=n // 10, count=n, qps=qps / fronts, threads=a.open_loop_threads,
                                  timeout_us=timeout_us)
            ach = n / (q["window_us"] * 1e-6) * fronts if q.get("window_us") else 0.0
            red = torch.tensor([pct(q["latency_us"], 50) or 0.0, pct(q["latency_us"], 99) or 0.0,
                                float(q["errors"]), -ach], dtype=torch.float64)
            if ctx.is_distributed:  # slowest front door's percentiles, lowest achieved rate
                dist.all_reduce(red, op=dist.ReduceOp.MAX, group=phase)
            sweep.append({"load": f, "offered_qps": round(qps, 1), "achieved_qps": round(-float(red[3]), 1),
                          "scores_per_s": round(qps * a.request_rows, 1), "p50_ms": round(float(red[0]), 3),
                          "p99_ms": round(float(red[1]), 3), "errors": int(red[2]), "stages": stage_breakdown(q)})
        extra["latency_vs_load"] = {"capacity_qps": round(cap_qps, 1), "request_rows": a.request_rows,
                                    "front_doors": fronts, "points": sweep,
                                    # this rank's host over the sweep: cgroup throttling, CPU use, preemptions
                                    "host": host_sched_delta(hs0, host_sched_counters())}
    # BASELINE config 2 literally: one 512-candidate request at a time (at N > 1
    # fanned out over every GPU: the reference's topology inside one node)
    sync()
    if rank == 0 and pool:
        c1 = live.run_load(pool, warmup=20, count=300, concurrency=1, threads=1, timeout_us=timeout_us)
        w = c1["window_us"] * 1e-6
        extra["config2_batch512"] = {"concurrency": 1, "p50_ms": pct(c1["latency_us"], 50),
                                     "p99_ms": pct(c1["latency_us"], 99),
                                     "scores_per_s": round(300 * a.request_rows / w, 1) if w > 0 else None}
    sync()
    st = live.stats()
    keys = ("steps", "full_steps", "timeout_steps", "eager_steps", "empty_steps", "proposed_steps", "joined_steps",
            "blocked_submits", "narrowed", "narrowed_wts_bf16", "narrowed_wts_implicit")
    extra["server"] = {k: st[k] for k in keys}
    extra["server"]["steps_in_throughput_run"] = st_load["steps"]
    if control is not None:
        # an idle cluster launches nothing: no step between the phases' ends
        t0 = st["steps"]
        time.sleep(0.05)
        extra["server"]["idle_steps_per_s"] = round((live.stats()["steps"] - t0) / 0.05, 1)
    extra["ingest"] = ("host-narrowed 3-byte / int32 rows + weights in their cheapest exact form (fp32, bf16, or none "
                       "when all 1.0; K0 on the submitting thread)" if live.narrow_modulo
                       else "raw request bytes, unpacked on the GPU")
    if hasattr(model, "exchange_bytes"):  # sharded tables: the embedding exchange of one step, per rank
        extra["embedding_exchange"] = {
            "bytes_per_step_per_rank": int(model.exchange_bytes(B)),
            "plan": {"world": model.plan.world, "row_wise_tables": len(model.plan.row_wise()),
                     "tables_per_rank": [len(model.plan.table_wise(r)) for r in range(model.plan.world)]},
            "multi_hot": int(getattr(model, "hot", 1)),
            "mode": model.emb.exchange,
            "hot_row_cache": None,
        }
        if cache is not None:
            hits, misses = cache_counts  # counted on every sample_every-th candidate
            steps = max(1, st_load["steps"] - steps0)
            lookups_per_step = (hits + misses) * cache.count_scale / steps
            extra["embedding_exchange"]["hot_row_cache"] = {
                **cache.describe(),
                "hits": hits, "misses": misses, "hit_rate": round(hits / max(1, hits + misses), 4),
                # measured over the throughput run (warmup + timed steps)
                "remote_lookups_per_step": round(lookups_per_step, 1),
                "xgmi_bytes_per_step_per_rank": int(misses * cache.count_scale / steps * cfg.embed_dim * 2),
                "counted_every": cache.count_scale,
                # the pool repeats: the same hot set on a fresh draw of the stream
                "hit_rate_fresh_stream": fresh_hit_rate(cfg, model, ctx),
                # exact top-k of the served pool's remote-key frequencies: the best
                # any hot set of k rows can do on this stream
                "oracle": cache_oracle(a, cfg, model, ctx, len(pool), [cache.cap, int(cache.keys.numel())]),
            }
    if eng.scatter is not None:
        # shared-arena scatter: host->device bytes this rank copied per step (its
        # share of rank 0's batch), gathered from every rank
        per = torch.tensor([float(eng.scatter.h2d_bytes) / max(1, eng.scatter.h2d_steps)], dtype=torch.float64)
        allp = [torch.zeros_like(per) for _ in range(world)]
        dist.all_gather(allp, per, group=phase)
        extra["scatter"] = {"path": "shared arena (each GPU DMAs its own share over its own link)",
                            "h2d_bytes_per_step_by_rank": [int(x.item()) for x in allp]}
    try:
        from distributed_tf_serving_amd.utils.affinity import placement

        extra["numa"] = placement()
    except Exception:  # noqa: BLE001 - informational only
        pass
    if a.json_extra and rank == 0:
        per = {k: round(st[k] / max(1, st["steps"]), 1) for k in ("copy_us", "build_us", "launch_us", "wait_us",
                                                                  "encode_us")}
        print(json.dumps({"server_us_per_step": per, "stats": st}), file=sys.stderr, flush=True)
    if cache is not None:
        cache.stop()  # the background refresher (--cache-refresh-s)
    live.close()  # cluster: returns once every rank has closed
    sync()
    return window_s, extra


def run_reference_over_grpc(a, live, cfg) -> dict:
    """The reference workload over the network: this process serves the native
    gRPC front door (csrc/net/h2_server.cpp) on the live server; a child
    process of native h2c clients (client/native_load.py, no GPU) runs the
    reference's closed loop against it over TCP (reference DCNClient.java:
    111-112, 205-241)."""
    import subprocess

    from distributed_tf_serving_amd.serving.native_front import NativeGrpcFront

    front = NativeGrpcFront(None, live, port=0, host="127.0.0.1", threads=a.grpc_threads)
    cmd = [sys.executable, "-m", "distributed_tf_serving_amd.client.native_load", "--port", str(front.port),
           "--candidates", str(a.request_rows), "--concurrency", str(a.ref_clients), "--requests",
           str(a.ref_requests), "--warmup", "10", "--id-mode", "reference", "--timeout-s", str(a.step_timeout_s)]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    try:
        p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    finally:
        st = front.stats()
        front.stop()
    line = next((ln for ln in p.stdout.splitlines() if ln.startswith("{")), None)
    if p.returncode != 0 or line is None:
        raise SystemExit(f"native gRPC clients failed ({p.returncode}): {p.stdout[-2000:]} {p.stderr[-2000:]}")
    res = json.loads(line)
    print(next(ln for ln in p.stdout.splitlines() if ln.startswith("Average")), flush=True)
    return {"metric": "reference workload (DCNClient.java) over gRPC: average request latency",
            "value": round(res["avg_ms"], 4), "unit": "ms", "higher_is_better": False, "n_gpus": 1,
            "requests": res["requests"], "errors": res["errors"], "clients": a.ref_clients,
            "candidates": a.request_rows, "p50_ms": round(res["p50_ms"], 4), "p99_ms": round(res["p99_ms"], 4),
            "requests_per_s": res["requests_per_s"], "scores_per_s": res["scores_per_s"],
            "front_door": {k: st[k] for k in ("connections", "calls", "replies", "protocol_errors", "bytes_in")},
            "path": "native h2c clients (separate process) -> TCP -> native gRPC front door -> live server (1 GPU)",
            "model": describe_model(cfg), "encoding": "int64_val / float_val (like the reference client)"}


def run_reference(a, ctx, cfg, model, eng, B):
    """--reference-workload: the reference client's closed loop against this
    server (reference DCNClient.java:205-241): ``--ref-clients`` threads x
    ``--ref-requests`` back-to-back 1500-candidate requests, latency per
    request from submit to the serialized PredictResponse, average printed
    in the reference's format."""
    world, rank, dev = ctx.world, ctx.rank, ctx.device
    pool, _ = request_pool(a, ctx, eng, B, cfg.num_fields)
    buckets = list(eng.ex.buckets)
    sc = ServingConfig(max_batch_rows=B, allowed_batch_sizes=tuple(buckets), batch_timeout_us=a.batch_timeout_us,
                       max_queued_rows=1 << 24, max_request_rows=1 << 20, model_name="DCN")
    control = None
    if eng.lockstep and world > 1:
        from distributed_tf_serving_amd.ops import hip
        from distributed_tf_serving_amd.parallel.control import control_for_job

        control = control_for_job(hip() if dev.type == "cuda" else native(), ctx, "bench-ref")
    live = LiveScheduler(eng, sc, buckets=buckets, depth=a.slots, control=control, step_timeout_s=a.step_timeout_s,
                         start_paused=control is not None, narrow=not a.no_narrow, peer_timeout_s=a.step_timeout_s)
    phase = dist.new_group(backend="gloo") if ctx.is_distributed else None
    tune_for_serving()
    if ctx.is_distributed:
        dist.barrier(group=phase)
    if control is not None:
        live.resume()
    out = None
    if pool and a.over_grpc:
        if world > 1:
            raise SystemExit("--over-grpc runs on one GPU (the front door of a cluster is serving/cluster.py)")
        out = run_reference_over_grpc(a, live, cfg)
        pool = None
    if pool:
        n = a.ref_clients * a.ref_requests
        r = live.run_load(pool, warmup=10 * a.ref_clients, count=n, concurrency=a.ref_clients,
                          threads=a.ref_clients, timeout_us=int(a.step_timeout_s * 1e6))
        lat_ms = [x * 1e-3 for x in r["latency_us"]]
        if a.print_requests:
            for i, ms in enumerate(lat_ms):
                print(f"Thread Thread-{i % a.ref_clients}. Time cost with {a.request_rows} is {ms} ms")
        avg = sum(lat_ms) / len(lat_ms) if lat_ms else float("nan")
        print(f"Average time cost with {a.request_rows} is {avg} ms with {len(lat_ms)} requests", flush=True)
        wall = r["wall_us"] * 1e-6
        st = live.stats()
        out = {"metric": "reference workload (DCNClient.java): average request latency", "value": round(avg, 4),
               "unit": "ms", "higher_is_better": False, "n_gpus": world, "requests": len(lat_ms),
               "errors": int(r["errors"]), "clients": a.ref_clients, "candidates": a.request_rows,
               "p50_ms": pct(r["latency_us"], 50), "p99_ms": pct(r["latency_us"], 99),
               "requests_per_s": round(len(lat_ms) / wall, 1) if wall > 0 else None,
               "scores_per_s": round(len(lat_ms) * a.request_rows / wall, 1) if wall > 0 else None,
               "steps": st["steps"], "buckets": buckets,
               "path": "in-process native clients -> live server" + (f" -> {eng.mode} over {world} GPUs"
                                                                      if world > 1 else " (1 GPU)"),
               "model": describe_model(cfg), "encoding": "int64_val / float_val (like the reference client)"}
    live.close()
    if ctx.is_distributed:
        dist.barrier(group=phase)
    if out is not None and rank == 0:
        print(json.dumps(out), flush=True)


def main():
    a = parse_args()
    if os.environ.get("DTFS_HANG_DUMP_S"):  # debugging aid: every thread's stack, then exit
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["DTFS_HANG_DUMP_S"]), exit=True)
    os.environ.setdefault("DTFS_HOST_THREADS", str(max(1, a.decode_threads)))
    if a.peer_comm is not None:
        os.environ["DTFS_PEER_COMM"] = str(max(0, a.peer_comm))  # read by parallel/native_comm.create_comm
    ctx = init_from_env()
    world, rank = ctx.world, ctx.rank
    if world != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = ctx.device
    torch.manual_seed(1234)
    cfg, model, eng, B = build(a, ctx)
    if a.reference_workload:
        run_reference(a, ctx, cfg, model, eng, B)
        shutdown()
        return
    el, extra = run_live(a, ctx, cfg, model, eng, B)

    t = torch.tensor([el, float(extra.get("requests_failed", 0))], dtype=torch.float64,
                     device=dev if ctx.backend == "nccl" else "cpu")
    if ctx.is_distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el_max, failed = float(t[0].item()), int(t[1].item())
    if failed:
        # a failed request means a server broke mid-run: the window no longer
        # measures served scores, so no number is reported (every rank agrees)
        if rank == 0:
            print(f"error: requests failed during the timed run; no result", file=sys.stderr, flush=True)
        shutdown()
        raise SystemExit(3)
    total_scores = world * B * a.steps
    value = total_scores / el_max if el_max > 0 else 0.0
    if rank == 0:
        if eng.mode == "local":
            par = f"candidate-dp{world} (" + ("one GPU, no fan-out" if world == 1 else
                                              "one independent replica per GPU, no collectives") + ")"
        elif eng.scatter is not None:
            par = (f"candidate-dp{world} (scatter fan-out through rank 0's shared request arenas: every GPU DMAs "
                   f"its own share, scores written into rank 0's shared output; "
                   + ("native C++ step" if dev.type == "cuda" else "host reference (CPU)") + ")")
        else:
            par = (f"candidate-dp{world} ({eng.mode} fan-out over RCCL"
                   + (", native C++ step" if eng.native_fanout_active else ", gloo (CPU)")
                   + (f", one-shot peer exchange for messages <= {eng._cin.peer_cap} B per peer"
                      if getattr(eng, "_cin", None) is not None and eng._cin.peer_enabled else "")
                   + (f", {eng.layout.row_bytes} B rows: int32 table rows + fp32 weights" if eng.layout.narrow
                      else f", {eng.layout.row_bytes} B rows: raw int64 ids + fp32 weights") + ")")
        if hasattr(model, "plan") and getattr(model.emb, "exchange", "") == "peer" and model.plan.world > 1:
            par += (f" + embedding-mp{model.plan.world} (table-wise, rows loaded from the owner's HBM over xGMI, "
                    + (f"{model.cache.cap}-row hot-row replica cache per rank" if model.cache is not None
                       else "no replica cache") + ")")
        elif hasattr(model, "plan"):
            par += (f" + embedding-mp{model.plan.world} ({len(model.plan.row_wise())} row-wise tables, all-to-all; "
                    + ("native two-lane step program" if eng.program_active else "eager torch.distributed")
                    + (f", one-shot peer exchange for messages <= {eng._cprog.peer_cap} B per peer"
                       if getattr(eng, "_cprog", None) is not None and eng._cprog.peer_enabled else "") + ")")
        out = {
            "metric": "CTR scores/sec (whole node)",
            "value": round(value, 1),
            "unit": "scores/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "prime_steps": a.prime_steps,
            "ms_per_step": round(el_max / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(value / BASELINE_VALUE, 4),
            "dtype": dtype_label(cfg),
            "data": ("synthetic (zipf feature ids over 2^40, " +
                     ("feature weights 1.0 as the reference client sends them" if a.feature_weights == "ones"
                      else "uniform weights") + "; random-init weights)"),
            "config": {
                "model": describe_model(cfg),
                "global_batch": world * B,
                "request_rows": a.request_rows,
                "requests_per_gpu_per_step": a.requests_per_gpu,
                "buckets": list(eng.ex.buckets),
                "seq_len": None,
                "parallelism": par,
                "encoding": a.encoding,
                "path": ("served: native live server (batching, arena copy, parse, step, encode) driven by "
                         "in-process native client threads"),
                # steps run as a two-lane program (fan-out: resolve pass on the ingress lane)
                "two_lane_buckets": sorted(set(eng._program_buckets) | {k[0] for k, v in eng._split.items() if v}),
                # CUs of the program's aux lane (0: unmasked; step_runner.cpp ensure_aux_stream)
                "aux_lane_cus": int(getattr(getattr(eng, "_runner", None), "aux_cus", 0) or 0),
            },
        }
        out.update(extra)
        print(json.dumps(out), flush=True)
    shutdown()


if __name__ == "__main__":
    main()

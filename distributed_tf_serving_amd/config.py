"""Configuration: dataclasses + YAML presets + argparse.

Every hard-coded knob of the reference client becomes a flag whose default is
the reference value (reference DCNClient.java:25-42):

=====================  ==================  ==============================
flag                   default             reference
=====================  ==================  ==============================
--fields               43                  FIELD_NUM            (:25)
--full-async / --poll  full async (A)      isFullAsyncMode      (:27)
--port                 9999                port                 (:28)
--candidates           1500                candidateNum         (:29)
--requests             1000                requestNum           (:30)
--concurrency          6                   concurrentNum        (:31)
--model-name           DCN                 modelName            (:33)
--signature            serving_default     modelSignature       (:34)
--output-key           prediction_node     outputKey            (:35)
--backends             3                   hostsList.size()     (:38)
--pool-threads         16                  newFixedThreadPool   (:42)
=====================  ==================  ==============================
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRESET_DIR = os.path.join(REPO, "configs")


@dataclass
class ModelConfig:
    """Architecture of one CTR model (random-init weights; see models/)."""

    family: str = "deepfm"            # wdl | deepfm | dcn | dcn_v2 | dlrm
    num_fields: int = 43              # reference FIELD_NUM
    vocab_size: int = 1_000_000       # rows of the shared table (wdl/deepfm/dcn/dcn_v2)
    embed_dim: int = 64
    mlp_dims: Tuple[int, ...] = (1024, 512, 256)
    num_cross_layers: int = 3         # dcn / dcn_v2
    cross_rank: int = 0               # dcn_v2: 0 = full-rank W, >0 = low-rank U V^T
    num_dense: int = 13               # dlrm: leading fields carried as dense values
    bottom_mlp: Tuple[int, ...] = (512, 256, 64)   # dlrm bottom MLP (last = embed_dim)
    table_rows: int = 1_000_000       # dlrm: rows per sparse table
    multi_hot: int = 1                # dlrm: ids per sparse table (> 1: weighted sum-pooled bag, K1b)
    # dlrm tables sharded over ranks: "alltoall" (ids + rows through RCCL),
    # "peer" (rows loaded from the owner's HBM over xGMI, hot remote rows from a
    # per-rank replica cache of hot_cache_rows rows - -1: a quarter of the
    # free device memory, capped at the remote rows; 0: no cache;
    # parallel/hot_cache.py) or
    # "auto" (peer on GPUs that can all load from each other, else alltoall)
    embedding_exchange: str = "auto"
    hot_cache_rows: int = -1
    param_dtype: str = "bf16"         # storage dtype of embeddings + dense weights
    gemm_dtype: str = "bf16"          # bf16 | fp8 (dcn_v2 towers on CDNA4 fp8 MFMA)
    seed: int = 1234

    @property
    def num_sparse(self) -> int:
        """Sparse tables (dlrm: the fields after the dense ones, ``multi_hot`` per table)."""
        if self.family == "dlrm":
            return (self.num_fields - self.num_dense) // max(1, self.multi_hot)
        return self.num_fields


@dataclass
class ServingConfig:
    """Model-server side (TF-Serving ModelServer equivalent)."""

    model_name: str = "DCN"
    signature_name: str = "serving_default"
    version: int = 1
    ids_key: str = "feat_ids"
    wts_key: str = "feat_wts"
    output_key: str = "prediction_node"
    max_batch_rows: int = 8192        # dynamic batcher: rows per GPU batch
    batch_timeout_us: int = 200       # oldest request waits at most this long
    hot_cache_refresh_s: float = 1.0  # peer-exchange DLRM: replica cache refresh period
    max_queued_rows: int = 1 << 22    # backpressure bound (rows)
    max_request_rows: int = 1 << 18   # one request's candidates (checked before any allocation)
    allowed_batch_sizes: Tuple[int, ...] = (512, 1024, 2048, 4096, 8192)  # padding buckets (HIP graphs)
    num_batch_threads: int = 1
    use_graphs: bool = True           # capture each bucket's forward in a HIP graph
    device: str = "auto"              # auto | cpu | cuda
    request_timeout_s: float = 10.0
    live: bool = True                 # native live server (csrc/runtime/live_server.h); False: Python scheduler
    step_timeout_s: float = 10.0      # a GPU step that takes longer marks the server broken (UNAVAILABLE)
    peer_timeout_s: float = 5.0       # multi-rank: a rank silent this long (no heartbeat) breaks the cluster
    # scatter mode on one node: "shared" = every rank DMAs its share of rank 0's
    # shared request arenas (csrc/runtime/shared_scatter.h); "rccl" = RCCL scatter
    scatter_path: str = "shared"
    narrow_ingest: bool = True        # GPU live server: int64 ids -> 3-byte / int32 table rows on the host (fp32 weights)


@dataclass
class ClientConfig:
    """Client / load generator (reference DCNClient.main)."""

    fields: int = 43
    candidates: int = 1500
    requests: int = 1000
    concurrency: int = 6
    pool_threads: int = 16
    backends: int = 3
    hosts: List[str] = field(default_factory=lambda: ["127.0.0.1"])
    port: int = 9999
    full_async: bool = True           # mode A (ordered join) vs mode B (completion order)
    model_name: str = "DCN"
    signature_name: str = "serving_default"
    output_key: str = "prediction_node"
    sort_scores: bool = True          # reference Collections.sort (DCNClient.java:195)
    id_mode: str = "reference"        # reference (ids 1..F, wts 1.0) | uniform | zipf
    id_space: int = 1_000_000
    zipf_a: float = 1.1
    raw_tensors: bool = False         # tensor_content instead of int64_val/float_val
    warmup: int = 0
    qps: float = 0.0                  # >0: open-loop fixed-QPS mode
    deadline_s: float = 0.0           # per-request deadline (0 = none)
    seed: int = 0


@dataclass
class Config:
    model: ModelConfig = field(default_factory=ModelConfig)
    serving: ServingConfig = field(default_factory=ServingConfig)
    client: ClientConfig = field(default_factory=ClientConfig)
    name: str = "default"
    description: str = ""


def _merge(dc, d: dict):
    for k, v in (d or {}).items():
        if not hasattr(dc, k):
            raise KeyError(f"unknown config key {type(dc).__name__}.{k}")
        cur = getattr(dc, k)
        if dataclasses.is_dataclass(cur):
            _merge(cur, v)
        else:
            if isinstance(cur, tuple) and isinstance(v, list):
                v = tuple(v)
            setattr(dc, k, v)
    return dc


def load_preset(name_or_path: str) -> Config:
    """Load configs/<name>.yaml (or a path) over the defaults (yaml.safe_load)."""
    path = name_or_path
    if not os.path.exists(path):
        path = os.path.join(PRESET_DIR, name_or_path + ".yaml")
    with open(path) as f:
        d = yaml.safe_load(f) or {}
    cfg = Config()
    cfg.name = d.pop("name", os.path.splitext(os.path.basename(path))[0])
    cfg.description = d.pop("description", "")
    return _merge(cfg, d)


def list_presets() -> List[str]:
    return sorted(os.path.splitext(f)[0] for f in os.listdir(PRESET_DIR) if f.endswith(".yaml"))


def to_dict(cfg) -> dict:
    return dataclasses.asdict(cfg)


def add_client_args(ap: argparse.ArgumentParser) -> None:
    c = ClientConfig()
    ap.add_argument("--fields", type=int, default=c.fields)
    ap.add_argument("--candidates", type=int, default=c.candidates)
    ap.add_argument("--requests", type=int, default=c.requests)
    ap.add_argument("--concurrency", type=int, default=c.concurrency)
    ap.add_argument("--pool-threads", type=int, default=c.pool_threads)
    ap.add_argument("--backends", type=int, default=c.backends)
    ap.add_argument("--hosts", type=str, default=None, help="comma-separated host[:port] list (grpc transport)")
    ap.add_argument("--port", type=int, default=c.port)
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--full-async", dest="full_async", action="store_true", default=True)
    g.add_argument("--poll", dest="full_async", action="store_false", help="mode B: completion-order gather")
    ap.add_argument("--model-name", default=c.model_name)
    ap.add_argument("--signature", default=c.signature_name)
    ap.add_argument("--output-key", default=c.output_key)
    ap.add_argument("--no-sort", dest="sort_scores", action="store_false", default=True)
    ap.add_argument("--id-mode", choices=["reference", "uniform", "zipf"], default=c.id_mode)
    ap.add_argument("--id-space", type=int, default=c.id_space)
    ap.add_argument("--raw-tensors", action="store_true")
    ap.add_argument("--warmup", type=int, default=c.warmup)
    ap.add_argument("--qps", type=float, default=c.qps)
    ap.add_argument("--deadline-s", type=float, default=c.deadline_s)
    ap.add_argument("--seed", type=int, default=c.seed)


def client_from_args(a) -> ClientConfig:
    c = ClientConfig(
        fields=a.fields, candidates=a.candidates, requests=a.requests, concurrency=a.concurrency,
        pool_threads=a.pool_threads, backends=a.backends, port=a.port, full_async=a.full_async,
        model_name=a.model_name, signature_name=a.signature, output_key=a.output_key,
        sort_scores=a.sort_scores, id_mode=a.id_mode, id_space=a.id_space, raw_tensors=a.raw_tensors,
        warmup=a.warmup, qps=a.qps, deadline_s=a.deadline_s, seed=a.seed)
    if getattr(a, "hosts", None):
        c.hosts = [h.strip() for h in a.hosts.split(",") if h.strip()]
    return c

"""Checkpoint / resume of servable weights.

The reference client has no state; the TF-Serving host it talks to loads a
SavedModel (reference DCNClient.java:33 model "DCN"; saver.proto / meta_graph.proto
are vendored only as imports). BASELINE asks for random-init weights, so
checkpoints here exist to pin a model: a deterministic seed plus a saved
state give identical scores on any number of GPUs.

Format: safetensors only (no pickle anywhere, so loading executes nothing from
the file).

* ``save_model`` / ``load_model``: one file, the module's state_dict, with
  the ModelConfig in the metadata.
* ``save_sharded`` / ``load_sharded`` (``ShardedDLRM``): one file per rank with
  that rank's table shards keyed by (table, first global row), plus the dense
  towers on rank 0, and a JSON manifest of every shard. Loading re-slices rows
  from whichever files hold them, so a checkpoint written by N ranks loads on
  M ranks (re-sharding).
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Dict, List, Optional

import torch
from safetensors import safe_open
from safetensors.torch import load_file, save_file

from ..config import ModelConfig

MANIFEST = "manifest.json"


def _cfg_meta(cfg: ModelConfig) -> Dict[str, str]:
    return {"model_config": json.dumps(dataclasses.asdict(cfg))}


def config_from_meta(meta: Dict[str, str]) -> ModelConfig:
    d = json.loads(meta["model_config"])
    for k, v in d.items():
        if isinstance(v, list):
            d[k] = tuple(v)
    return ModelConfig(**d)


def _state(module: torch.nn.Module) -> Dict[str, torch.Tensor]:
    # parameters + buffers (fp8 weight copies included), contiguous CPU copies
    return {k: v.detach().contiguous().cpu() for k, v in module.state_dict().items()}


def save_model(model: torch.nn.Module, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    save_file(_state(model), path, metadata=_cfg_meta(model.cfg))


def load_model(model: torch.nn.Module, path: str, strict: bool = True) -> torch.nn.Module:
    sd = load_file(path, device=str(next(model.parameters()).device))
    model.load_state_dict(sd, strict=strict)
    return model


def read_config(path: str) -> ModelConfig:
    with safe_open(path, "pt") as f:
        return config_from_meta(f.metadata())


# ---------------------------------------------------------------- sharded DLRM
def _shard_key(table: int, lo: int) -> str:
    return f"table{table}.rows{lo}"


def save_sharded(model, path: str) -> None:
    """Collective over the model's process group: every rank writes its file."""
    import torch.distributed as dist

    emb = model.emb
    rank, world = emb.rank, emb.world
    os.makedirs(path, exist_ok=True)
    tensors, shards = {}, []
    for t, lo, n, off in emb.segments:
        if n == 0:
            continue
        tensors[_shard_key(t, lo)] = emb.store[off:off + n].detach().contiguous().cpu()
        shards.append({"table": t, "lo": lo, "rows": n, "file": f"rank{rank}.safetensors"})
    if rank == 0:
        for k, v in _state(model.dense).items():
            tensors["dense." + k] = v
    save_file(tensors, os.path.join(path, f"rank{rank}.safetensors"), metadata=_cfg_meta(model.cfg))
    all_shards: List = [None] * world
    if world > 1 and dist.is_initialized():
        dist.all_gather_object(all_shards, shards)
    else:
        all_shards = [shards]
    if rank == 0:
        manifest = {"world": world, "shards": [s for part in all_shards for s in part],
                    "model_config": json.loads(_cfg_meta(model.cfg)["model_config"])}
        with open(os.path.join(path, MANIFEST), "w") as f:
            json.dump(manifest, f, indent=1)
    if world > 1 and dist.is_initialized():
        dist.barrier()


def load_sharded(model, path: str) -> None:
    """Fill this rank's shards (any saved world size) and the dense towers."""
    with open(os.path.join(path, MANIFEST)) as f:
        manifest = json.load(f)
    by_table: Dict[int, List[dict]] = {}
    for s in manifest["shards"]:
        by_table.setdefault(s["table"], []).append(s)
    emb = model.emb
    handles: Dict[str, object] = {}

    def h(fname):
        if fname not in handles:
            handles[fname] = safe_open(os.path.join(path, fname), "pt")
        return handles[fname]

    with torch.no_grad():
        for t, lo, n, off in emb.segments:
            need_lo, need_hi = lo, lo + n
            filled = 0
            for s in sorted(by_table.get(t, []), key=lambda s: s["lo"]):
                a, b = max(need_lo, s["lo"]), min(need_hi, s["lo"] + s["rows"])
                if a >= b:
                    continue
                rows = h(s["file"]).get_slice(_shard_key(t, s["lo"]))[a - s["lo"]:b - s["lo"]]
                emb.store[off + a - lo:off + b - lo].copy_(rows)
                filled += b - a
            if filled != n:
                raise ValueError(f"checkpoint covers {filled} of table {t}'s rows [{lo}, {lo + n})")
        f0 = h("rank0.safetensors")
        dense = {k[len("dense."):]: f0.get_tensor(k) for k in f0.keys() if k.startswith("dense.")}
        model.dense.load_state_dict(dense, strict=True)

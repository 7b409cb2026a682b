"""Synthetic candidate features (there is no dataset in this environment).

Modes:

``reference``  exactly the reference workload: every candidate has ids 1..F
               and weights 1.0 (reference DCNClient.java:57-74). Perfect
               cache locality - kept for diff-ability with the reference.
``uniform``    ids uniform over ``id_space``.
``zipf``       per-field Zipf(a) popularity over ``id_space`` (realistic CTR
               skew: a few hot ids, a long tail), weights uniform in (0, 1].

``weights="ones"`` gives the uniform / zipf modes the reference client's
feature weights (every one 1.0, DCNClient.java:67-73) instead.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from ..wire import schema as pb
from ..wire.tensor import make_tensor_proto

_GOLD = np.uint64(0x9E3779B97F4A7C15)


class SyntheticRequests:
    def __init__(self, fields: int = 43, id_space: int = 1_000_000, dist: str = "zipf", zipf_a: float = 1.1,
                 seed: int = 0, model_name: str = "DCN", signature_name: str = "serving_default",
                 ids_key: str = "feat_ids", wts_key: str = "feat_wts", weights: str = "uniform"):
        if dist not in ("reference", "uniform", "zipf"):
            raise ValueError(f"unknown id distribution {dist!r}")
        if weights not in ("uniform", "ones"):
            raise ValueError(f"unknown feature weights {weights!r}")
        self.weights = weights
        self.F, self.space, self.dist, self.a = fields, int(id_space), dist, zipf_a
        self.rng = np.random.default_rng(seed)
        self.model_name, self.signature_name = model_name, signature_name
        self.ids_key, self.wts_key = ids_key, wts_key

    def arrays(self, rows: int) -> Tuple[np.ndarray, np.ndarray]:
        F = self.F
        if self.dist == "reference":
            ids = np.tile(np.arange(1, F + 1, dtype=np.int64), (rows, 1))
            return ids, np.ones((rows, F), dtype=np.float32)
        if self.dist == "uniform":
            ids = self.rng.integers(0, self.space, size=(rows, F), dtype=np.int64)
        else:
            rank = self.rng.zipf(self.a, size=(rows, F)).astype(np.uint64)
            # scatter popularity ranks over the id space, differently per field
            field_salt = (np.arange(F, dtype=np.uint64) + np.uint64(1)) * np.uint64(0x632BE59BD9B4E019)
            with np.errstate(over="ignore"):
                h = (rank * _GOLD) ^ field_salt[None, :]
            ids = (h % np.uint64(self.space)).astype(np.int64)
        if self.weights == "ones":
            return ids, np.ones((rows, F), dtype=np.float32)
        wts = self.rng.random((rows, F), dtype=np.float32)
        wts = np.where(wts == 0, np.float32(1.0), wts)
        return ids, wts

    def message(self, rows: int, raw: bool = False):
        ids, wts = self.arrays(rows)
        r = pb.PredictRequest()
        r.model_spec.name = self.model_name
        r.model_spec.signature_name = self.signature_name
        r.inputs[self.ids_key].CopyFrom(make_tensor_proto(ids, raw=raw))
        r.inputs[self.wts_key].CopyFrom(make_tensor_proto(wts, raw=raw))
        return r

    def serialized(self, rows: int, raw: bool = True) -> bytes:
        from ..ops import native

        ids, wts = self.arrays(rows)
        return native().encode_predict_request(
            self.model_name, self.signature_name, None,
            [(self.ids_key, torch.from_numpy(ids)), (self.wts_key, torch.from_numpy(wts))], raw)

"""Model registry: name -> versions -> servable, with TF-Serving's version policy.

``ModelSpec.version`` unset means "the highest loaded version" (reference
model.proto:13-14, predict.proto:13-15). ``signature_name`` empty means
``serving_default``. The reference talks to one SavedModel "DCN" with signature
"serving_default" (DCNClient.java:33-34); here any number of random-init CTR
models can be loaded side by side, each with its own batching scheduler.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .errors import Code, ServingError

DEFAULT_SIGNATURE = "serving_default"
PREDICT_METHOD = "tensorflow/serving/predict"
CLASSIFY_METHOD = "tensorflow/serving/classify"
REGRESS_METHOD = "tensorflow/serving/regress"


@dataclass
class Signature:
    inputs: Dict[str, tuple]      # key -> (dtype name, shape)
    outputs: Dict[str, tuple]
    method_name: str = PREDICT_METHOD


@dataclass
class Servable:
    name: str
    version: int
    model: object                              # CTRModel
    scheduler: object                          # BatchingScheduler
    signatures: Dict[str, Signature] = field(default_factory=dict)
    ids_key: str = "feat_ids"
    wts_key: str = "feat_wts"
    output_key: str = "prediction_node"
    fields: int = 43

    def signature(self, name: str) -> Signature:
        name = name or DEFAULT_SIGNATURE
        sig = self.signatures.get(name)
        if sig is None:
            raise ServingError(Code.INVALID_ARGUMENT,
                               f"Serving signature name: \"{name}\" not found in signature def of model {self.name}")
        return sig


class ModelRegistry:
    def __init__(self):
        self._models: Dict[str, Dict[int, Servable]] = {}
        self._lock = threading.Lock()

    def load(self, servable: Servable) -> None:
        with self._lock:
            self._models.setdefault(servable.name, {})[servable.version] = servable

    def replace(self, servable: Servable) -> Optional[Servable]:
        """Swap in a servable for the same (name, version); the previous one is
        returned, not closed (the caller drains it)."""
        with self._lock:
            vs = self._models.setdefault(servable.name, {})
            old = vs.get(servable.version)
            vs[servable.version] = servable
            return old

    def unload(self, name: str, version: Optional[int] = None) -> None:
        with self._lock:
            vs = self._models.get(name, {})
            for v in ([version] if version is not None else list(vs)):
                s = vs.pop(v, None)
                if s is not None and hasattr(s.scheduler, "close"):
                    s.scheduler.close()
            if not vs:
                self._models.pop(name, None)

    def only(self) -> Optional[Servable]:
        """The servable when exactly one (name, version) is loaded, else None."""
        models = self._models
        if len(models) != 1:
            return None
        vs = next(iter(models.values()))
        return next(iter(vs.values())) if len(vs) == 1 else None

    def names(self) -> List[str]:
        return sorted(self._models)

    def versions(self, name: str) -> List[int]:
        return sorted(self._models.get(name, {}))

    def resolve(self, name: str, version: Optional[int] = None) -> Servable:
        vs = self._models.get(name)
        if not vs:
            raise ServingError(Code.NOT_FOUND, f"Servable not found for request: Latest({name})")
        if version is None:
            return vs[max(vs)]
        s = vs.get(int(version))
        if s is None:
            raise ServingError(Code.NOT_FOUND, f"Servable not found for request: Specific({name}, {version})")
        return s

    def close(self) -> None:
        for name in list(self._models):
            self.unload(name)

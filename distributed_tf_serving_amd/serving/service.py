"""The PredictionService surface (reference prediction_service.proto:15-31).

All five RPCs are implemented against the model registry:

``Predict``          inputs feat_ids / feat_wts [B, F] -> outputs prediction_node [B]
                     (the only RPC the reference client calls, DCNClient.java:111-112);
                     on request (output_filter) also the RANKED outputs
                     sorted_prediction [B] (ascending, the reference client's
                     Collections.sort, DCNClient.java:195) and sorted_index [B]
                     (the candidate permutation the reference loses), computed
                     by the K7 bitonic sort kernel on the servable's GPU
``Classify``         tf.Example list -> per example {label "click", score}
``Regress``          tf.Example list -> per example CTR value
``MultiInference``   several classify/regress tasks over one Example list
``GetModelMetadata`` SignatureDefMap packed in Any (meta_graph.proto:297-311)

Predict has two entry points: :meth:`predict_bytes` (serialized request ->
serialized response, through the native zero-copy codec: the gRPC front door
and in-process clients use this) and :meth:`predict` (message objects,
through python protobuf + the numpy codec).
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..ops import native
from ..wire import schema as pb
from ..wire import tensor as T
from .errors import Code, ServingError
from .registry import CLASSIFY_METHOD, PREDICT_METHOD, REGRESS_METHOD, ModelRegistry, Servable

CLICK_LABEL = "click"
# ranked outputs: produced only when named in output_filter (an empty filter
# returns prediction_node alone - unlike TF's "all outputs" - so the hot path
# never pays for a sort)
SORTED_SCORES, SORTED_INDEX = "sorted_prediction", "sorted_index"
RANKED_OUTPUTS = (SORTED_SCORES, SORTED_INDEX)


def _dt(name: str) -> int:
    return pb.DataType[name]


class PredictionServiceImpl:
    def __init__(self, registry: ModelRegistry, default_timeout_s: float = 10.0):
        self.registry = registry
        self.timeout_s = default_timeout_s
        self.nat = native()

    # ------------------------------------------------------------------ helpers
    def _resolve(self, spec) -> Servable:
        version = spec.version.value if spec.HasField("version") else None
        return self.registry.resolve(spec.name, version)

    def _deadline_us(self, timeout_s: Optional[float]) -> int:
        t = self.timeout_s if timeout_s is None else timeout_s
        return int(self.nat.now_us() + t * 1e6) if t and t > 0 else 0

    def _wait(self, fut: cf.Future, timeout_s: Optional[float]):
        t = self.timeout_s if timeout_s is None else timeout_s
        try:
            return fut.result(timeout=t if t and t > 0 else None)
        except cf.TimeoutError:
            raise ServingError(Code.DEADLINE_EXCEEDED, "request timed out") from None

    def _spec_out(self, out_spec, s: Servable, sig_name: str) -> None:
        out_spec.name = s.name
        out_spec.version.value = s.version
        out_spec.signature_name = sig_name or "serving_default"

    def _check_filter(self, s: Servable, flt) -> None:
        for k in flt:
            if k != s.output_key and k not in RANKED_OUTPUTS:
                raise ServingError(Code.INVALID_ARGUMENT, f"output tensor alias not found in signature: {k}")

    def _outputs(self, s: Servable, flt, scores: torch.Tensor) -> List[Tuple[str, torch.Tensor]]:
        """(key, tensor) pairs of a Predict response: prediction_node unless the
        filter names only other outputs, plus the requested ranked outputs
        (K7 on the servable's device: ops.sort_scores)."""
        flt = list(flt)
        out = []
        if not flt or s.output_key in flt:
            out.append((s.output_key, scores))
        if any(k in RANKED_OUTPUTS for k in flt):
            from .. import ops

            dev = getattr(getattr(s.model, "device_", None), "type", "cpu")
            src = scores.to(s.model.device_) if dev == "cuda" else scores
            srt, perm = ops.sort_scores(src.float())
            if SORTED_SCORES in flt:
                out.append((SORTED_SCORES, srt.cpu()))
            if SORTED_INDEX in flt:
                out.append((SORTED_INDEX, perm.cpu().to(torch.int64)))
        return out

    # ------------------------------------------------------------------ Predict (bytes, native codec)
    def predict_async_bytes(self, data: bytes, timeout_s: Optional[float] = None) -> Tuple[cf.Future, object]:
        """Parse + enqueue; returns (future of scores, context for encode)."""
        try:
            req = self.nat.parse_predict_request(data)
        except ValueError as e:
            raise ServingError(Code.INVALID_ARGUMENT, str(e)) from None
        version = req.version
        s = self.registry.resolve(req.model_name, version)
        s.signature(req.signature_name)
        self._check_filter(s, req.output_filter)
        for key in (s.ids_key, s.wts_key):
            if not req.has_input(key):
                raise ServingError(Code.INVALID_ARGUMENT, f"input tensor alias not found in signature: {key}")
        shape = req.shape(s.ids_key)
        if len(shape) != 2 or shape[1] != s.fields:
            raise ServingError(Code.INVALID_ARGUMENT,
                               f"{s.ids_key} must have shape [B, {s.fields}], got {list(shape)}")
        if req.shape(s.wts_key) != shape:
            raise ServingError(Code.INVALID_ARGUMENT, f"{s.wts_key} shape {req.shape(s.wts_key)} != {list(shape)}")
        if req.dtype(s.ids_key) not in (pb.DT_INT64, pb.DT_INT32):
            raise ServingError(Code.INVALID_ARGUMENT, f"{s.ids_key} must be DT_INT64 or DT_INT32")
        rows = int(shape[0])

        flt = list(req.output_filter)

        def fill(ids_v, wts_v, req=req, s=s):
            req.decode_into(s.ids_key, ids_v, 0, 0)
            req.decode_into(s.wts_key, wts_v, 0, 0)

        fut = s.scheduler.submit(rows, fill, self._deadline_us(timeout_s))
        return fut, (s, req.signature_name, flt)

    def encode_predict(self, ctx, scores: torch.Tensor, raw: bool = False) -> bytes:
        s, sig = ctx[0], ctx[1]
        flt = ctx[2] if len(ctx) > 2 else ()
        return self.nat.encode_predict_response(s.name, sig or "serving_default", s.version,
                                                [(k, t.contiguous()) for k, t in self._outputs(s, flt, scores)], raw)

    def _live_fast(self):
        """The live scheduler when exactly one servable is loaded (the common
        case): serialized requests go straight to its native server, which
        validates model name / version / signature itself."""
        only = self.registry.only()
        sched = getattr(only, "scheduler", None) if only is not None else None
        return sched if sched is not None and hasattr(sched, "predict_raw") else None

    def predict_bytes(self, data: bytes, timeout_s: Optional[float] = None) -> bytes:
        live = self._live_fast()
        if live is not None:
            t = self.timeout_s if timeout_s is None else timeout_s
            code, msg, resp = live.predict_raw(data, t)
            if code == 0:
                return resp
            # NOT_FOUND / oversize / ranked outputs: the general path resolves, splits or sorts
            if code not in (Code.NOT_FOUND, live.OVERSIZE, live.CALLER_PATH):
                raise ServingError(Code(code) if code in Code._value2member_map_ else Code.UNKNOWN, msg)
        fut, ctx = self.predict_async_bytes(data, timeout_s)
        return self.encode_predict(ctx, self._wait(fut, timeout_s))

    # ------------------------------------------------------------------ Predict (messages)
    def predict(self, request, timeout_s: Optional[float] = None):
        s = self._resolve(request.model_spec)
        s.signature(request.model_spec.signature_name)
        self._check_filter(s, request.output_filter)
        try:
            ids = T.to_ndarray(request.inputs[s.ids_key]) if s.ids_key in request.inputs else None
            wts = T.to_ndarray(request.inputs[s.wts_key]) if s.wts_key in request.inputs else None
        except T.InvalidArgument as e:
            raise ServingError(Code.INVALID_ARGUMENT, str(e)) from None
        if ids is None or wts is None:
            raise ServingError(Code.INVALID_ARGUMENT, f"inputs {s.ids_key} and {s.wts_key} are required")
        scores = self._score(s, ids, wts, timeout_s)
        resp = pb.PredictResponse()
        self._spec_out(resp.model_spec, s, request.model_spec.signature_name)
        for key, t in self._outputs(s, request.output_filter, scores):
            resp.outputs[key].CopyFrom(T.make_tensor_proto(t.numpy()))
        return resp

    def _score(self, s: Servable, ids: np.ndarray, wts: np.ndarray, timeout_s=None) -> torch.Tensor:
        if ids.ndim != 2 or ids.shape[1] != s.fields or wts.shape != ids.shape:
            raise ServingError(Code.INVALID_ARGUMENT, f"expected [B, {s.fields}] inputs, got {ids.shape}/{wts.shape}")
        if not np.issubdtype(ids.dtype, np.integer):
            raise ServingError(Code.INVALID_ARGUMENT, f"{s.ids_key} must be an integer tensor")
        it = torch.from_numpy(np.ascontiguousarray(ids.astype(np.int64, copy=False)))
        wt = torch.from_numpy(np.ascontiguousarray(wts.astype(np.float32, copy=False)))

        def fill(iv, wv):
            iv.copy_(it)
            wv.copy_(wt)

        return self._wait(s.scheduler.submit(ids.shape[0], fill, self._deadline_us(timeout_s)), timeout_s)

    # ------------------------------------------------------------------ tf.Example based RPCs
    def _examples(self, s: Servable, inp) -> Tuple[np.ndarray, np.ndarray]:
        kind = inp.WhichOneof("kind")
        if kind is None:
            raise ServingError(Code.INVALID_ARGUMENT, "Input is empty")
        exs = inp.example_list.examples if kind == "example_list" else inp.example_list_with_context.examples
        ctx = inp.example_list_with_context.context if kind == "example_list_with_context" else None
        n = len(exs)
        ids = np.zeros((n, s.fields), dtype=np.int64)
        wts = np.ones((n, s.fields), dtype=np.float32)
        for i, ex in enumerate(exs):
            for key, arr, attr in ((s.ids_key, ids, "int64_list"), (s.wts_key, wts, "float_list")):
                feat = ex.features.feature.get(key)
                if feat is None and ctx is not None:
                    feat = ctx.features.feature.get(key)
                if feat is None:
                    if key == s.ids_key:
                        raise ServingError(Code.INVALID_ARGUMENT, f"example {i} has no feature {key}")
                    continue
                vals = list(getattr(feat, attr).value)
                if len(vals) != s.fields:
                    raise ServingError(Code.INVALID_ARGUMENT,
                                       f"example {i} feature {key} has {len(vals)} values, expected {s.fields}")
                arr[i] = vals
        return ids, wts

    def classify(self, request, timeout_s: Optional[float] = None):
        s = self._resolve(request.model_spec)
        s.signature(request.model_spec.signature_name)
        ids, wts = self._examples(s, request.input)
        scores = self._score(s, ids, wts, timeout_s) if len(ids) else torch.empty(0)
        resp = pb.ClassificationResponse()
        self._spec_out(resp.model_spec, s, request.model_spec.signature_name)
        self._fill_classification(resp.result, scores)
        return resp

    @staticmethod
    def _fill_classification(result, scores):
        for p in scores.tolist():
            c = result.classifications.add()
            cl = c.classes.add()
            cl.label = CLICK_LABEL
            cl.score = p

    def regress(self, request, timeout_s: Optional[float] = None):
        s = self._resolve(request.model_spec)
        s.signature(request.model_spec.signature_name)
        ids, wts = self._examples(s, request.input)
        scores = self._score(s, ids, wts, timeout_s) if len(ids) else torch.empty(0)
        resp = pb.RegressionResponse()
        self._spec_out(resp.model_spec, s, request.model_spec.signature_name)
        for p in scores.tolist():
            resp.result.regressions.add().value = p
        return resp

    def multi_inference(self, request, timeout_s: Optional[float] = None):
        if not request.tasks:
            raise ServingError(Code.INVALID_ARGUMENT, "MultiInferenceRequest has no tasks")
        resp = pb.MultiInferenceResponse()
        cache = {}
        for task in request.tasks:
            s = self._resolve(task.model_spec)
            s.signature(task.model_spec.signature_name)
            if task.method_name not in (CLASSIFY_METHOD, REGRESS_METHOD):
                raise ServingError(Code.UNIMPLEMENTED, f"unsupported method_name {task.method_name!r}")
            key = (s.name, s.version)
            if key not in cache:
                ids, wts = self._examples(s, request.input)
                cache[key] = self._score(s, ids, wts, timeout_s) if len(ids) else torch.empty(0)
            scores = cache[key]
            res = resp.results.add()
            self._spec_out(res.model_spec, s, task.model_spec.signature_name)
            if task.method_name == CLASSIFY_METHOD:
                self._fill_classification(res.classification_result, scores)
            else:
                for p in scores.tolist():
                    res.regression_result.regressions.add().value = p
        return resp

    def get_model_metadata(self, request):
        s = self._resolve(request.model_spec)
        fields = list(request.metadata_field)
        if fields != ["signature_def"]:
            raise ServingError(Code.INVALID_ARGUMENT, "Metadata field \"signature_def\" is the only supported field")
        sdm = pb.SignatureDefMap()
        for name, sig in s.signatures.items():
            sd = sdm.signature_def[name]
            sd.method_name = sig.method_name
            for key, (dt, shape) in sig.inputs.items():
                ti = sd.inputs[key]
                ti.name = f"{key}:0"
                ti.dtype = _dt(dt)
                ti.tensor_shape.CopyFrom(T.make_shape(shape))
            for key, (dt, shape) in sig.outputs.items():
                ti = sd.outputs[key]
                ti.name = f"{key}:0"
                ti.dtype = _dt(dt)
                ti.tensor_shape.CopyFrom(T.make_shape(shape))
        resp = pb.GetModelMetadataResponse()
        resp.model_spec.name = s.name
        resp.model_spec.version.value = s.version
        resp.metadata["signature_def"].Pack(sdm)
        return resp

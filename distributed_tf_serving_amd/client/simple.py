"""Smoke client (reference DCNClientSimple, DCNClientSimple.java:25-61).

Sends one Predict to host:port and prints the response. By default the request
is well-formed ([2, 43] with 86 ids/weights); ``--reference-shape`` reproduces
the reference exactly: shape [1500, 43] with only 87 ids and 86 weights, which
works only through TF's fill-with-last-value semantics (tensor.proto:24-29).
"""
from __future__ import annotations

import argparse

from ..wire import schema as pb
from ..wire.tensor import make_shape
from .backends import GrpcBackend


def build_request(reference_shape: bool = False, fields: int = 43, model: str = "DCN",
                  signature: str = "serving_default"):
    r = pb.PredictRequest()
    r.model_spec.name = model
    r.model_spec.signature_name = signature
    rows = 1500 if reference_shape else 2
    for key, dt in (("feat_ids", pb.DT_INT64), ("feat_wts", pb.DT_FLOAT)):
        t = r.inputs[key]
        t.dtype = dt
        t.tensor_shape.CopyFrom(make_shape([rows, fields]))
    r.inputs["feat_ids"].int64_val.extend(list(range(1, fields + 1)) +
                                          list(range(fields, 2 * fields + (1 if reference_shape else 0))))
    r.inputs["feat_wts"].float_val.extend([1.0] * (2 * fields))
    return r


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9999)
    ap.add_argument("--reference-shape", action="store_true")
    a = ap.parse_args(argv)
    be = GrpcBackend(f"{a.host}:{a.port}")
    try:
        resp = pb.PredictResponse.FromString(be.predict(build_request(a.reference_shape).SerializeToString(), 30))
        print(resp)
    finally:
        be.close()  # the reference never closes its channel (DCNClientSimple.java:54-60)


if __name__ == "__main__":
    main()

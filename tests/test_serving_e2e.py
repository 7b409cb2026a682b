"""End-to-end on CPU: ModelServer (Wide&Deep-tiny, BASELINE config 1) behind the
gRPC front door and in-process; fan-out client, load generator, all 5 RPCs,
error mapping."""
import io
import json

import grpc
import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.backends import GrpcBackend, InProcessBackend
from distributed_tf_serving_amd.client.fanout_client import FanoutClient, RequestSpec, ShardError
from distributed_tf_serving_amd.client.loadgen import LoadGenerator
from distributed_tf_serving_amd.client.simple import build_request
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.serving.errors import Code, ServingError
from distributed_tf_serving_amd.serving.server import ModelServer
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire import tensor as T


@pytest.fixture(scope="module")
def server():
    cfg = load_preset("wdl_tiny_cpu")
    cfg.serving.max_batch_rows = 64
    cfg.serving.allowed_batch_sizes = (1, 8, 64)
    cfg.serving.batch_timeout_us = 200
    srv = ModelServer(cfg, device="cpu")
    port = srv.start_grpc(0, "127.0.0.1")
    yield srv, port
    srv.stop()


def _expected(srv, ids, wts):
    m = srv.registry.resolve("DCN").model
    return m(torch.as_tensor(ids), torch.as_tensor(wts))


def test_predict_grpc_reference_request(server):
    srv, port = server
    be = GrpcBackend(f"127.0.0.1:{port}")
    try:
        req = build_request(reference_shape=True)  # DCNClientSimple: [1500,43], 87 ids
        resp = pb.PredictResponse.FromString(be.predict(req.SerializeToString(), 30))
        scores = T.to_ndarray(resp.outputs["prediction_node"])
        assert scores.shape == (1500,)
        assert resp.model_spec.name == "DCN" and resp.model_spec.version.value == 1
        ids = T.to_ndarray(req.inputs["feat_ids"])
        wts = T.to_ndarray(req.inputs["feat_wts"])
        assert np.allclose(scores, _expected(srv, ids, wts).numpy(), atol=1e-6)
    finally:
        be.close()


def test_fanout_client_modes(server):
    srv, port = server
    backends = [GrpcBackend(f"127.0.0.1:{port}") for _ in range(3)] + [InProcessBackend(srv.service)]
    rng = np.random.default_rng(0)
    ids = torch.from_numpy(rng.integers(0, 1 << 40, (187, 43)))
    wts = torch.rand(187, 43)
    exp = _expected(srv, ids, wts)
    for full_async in (True, False):
        cl = FanoutClient(backends, RequestSpec(raw=not full_async), pool_threads=16, full_async=full_async)
        res = cl.predict(ids, wts)
        if full_async:
            assert torch.allclose(res.scores, exp, atol=1e-6)
            assert torch.equal(res.sorted_scores, res.scores[res.order])
            assert res.shard_order == [0, 1, 2, 3]
        else:
            assert sorted(res.shard_order) == [0, 1, 2, 3]
            assert torch.allclose(torch.sort(res.scores).values, torch.sort(exp).values, atol=1e-6)
        cl.pool.shutdown()
    for b in backends:
        b.close()


def test_loadgen_reference_lines(server):
    srv, port = server
    cl = FanoutClient([InProcessBackend(srv.service) for _ in range(3)], pool_threads=16)
    out = io.StringIO()
    lg = LoadGenerator(cl, candidates=150, id_mode="reference", out=out)
    summary = lg.closed_loop(concurrency=3, requests=4, warmup=1)
    lines = out.getvalue().strip().splitlines()
    assert sum(l.startswith("Thread Thread-") and " Time cost with 150 is " in l for l in lines) == 12
    assert lines[-1].startswith("Average time cost with 150 is ") and lines[-1].endswith(" ms with 12 requests")
    assert summary["requests"] == 12 and summary["errors"] == 0 and summary["p50_ms"] > 0
    s2 = lg.open_loop(qps=200, total=10)
    assert s2["requests"] == 10
    json.dumps(summary)
    cl.close()


def test_errors_map_to_status(server):
    srv, port = server
    be = GrpcBackend(f"127.0.0.1:{port}")
    try:
        bad_model = build_request()
        bad_model.model_spec.name = "nope"
        with pytest.raises(grpc.RpcError) as e:
            be.predict(bad_model.SerializeToString(), 10)
        assert e.value.code() == grpc.StatusCode.NOT_FOUND
        bad_sig = build_request()
        bad_sig.model_spec.signature_name = "other"
        with pytest.raises(grpc.RpcError) as e:
            be.predict(bad_sig.SerializeToString(), 10)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        bad_shape = build_request()
        bad_shape.inputs["feat_ids"].tensor_shape.dim[1].size = 7
        with pytest.raises(grpc.RpcError) as e:
            be.predict(bad_shape.SerializeToString(), 10)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        with pytest.raises(grpc.RpcError) as e:
            be.predict(b"\xff\xff\xff", 10)
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        bad_ver = build_request()
        bad_ver.model_spec.version.value = 42
        with pytest.raises(grpc.RpcError) as e:
            be.predict(bad_ver.SerializeToString(), 10)
        assert e.value.code() == grpc.StatusCode.NOT_FOUND
    finally:
        be.close()
    cl = FanoutClient([GrpcBackend("127.0.0.1:1")], timeout_s=2)  # nothing listens on port 1
    with pytest.raises(ShardError):
        cl.predict(torch.zeros(2, 43, dtype=torch.int64), torch.ones(2, 43))
    cl.close()


def _examples(n, fields=43):
    inp = pb.Input()
    for i in range(n):
        ex = inp.example_list.examples.add()
        ex.features.feature["feat_ids"].int64_list.value.extend(range(i, i + fields))
        ex.features.feature["feat_wts"].float_list.value.extend([0.5] * fields)
    return inp


def test_classify_regress_multi_metadata(server):
    srv, port = server
    be = GrpcBackend(f"127.0.0.1:{port}")
    try:
        creq = pb.ClassificationRequest()
        creq.model_spec.name = "DCN"
        creq.input.CopyFrom(_examples(3))
        cres = be.call("Classify", creq, 10)
        ids = np.stack([np.arange(i, i + 43) for i in range(3)])
        exp = _expected(srv, ids, np.full((3, 43), 0.5, np.float32)).numpy()
        got = [c.classes[0].score for c in cres.result.classifications]
        assert np.allclose(got, exp, atol=1e-6) and cres.result.classifications[0].classes[0].label == "click"
        rreq = pb.RegressionRequest()
        rreq.model_spec.name = "DCN"
        rreq.input.CopyFrom(_examples(3))
        rres = be.call("Regress", rreq, 10)
        assert np.allclose([r.value for r in rres.result.regressions], exp, atol=1e-6)
        mreq = pb.MultiInferenceRequest()
        for m in ("tensorflow/serving/classify", "tensorflow/serving/regress"):
            t = mreq.tasks.add()
            t.model_spec.name = "DCN"
            t.method_name = m
        mreq.input.CopyFrom(_examples(2))
        mres = be.call("MultiInference", mreq, 10)
        assert len(mres.results) == 2 and mres.results[1].WhichOneof("result") == "regression_result"
        greq = pb.GetModelMetadataRequest()
        greq.model_spec.name = "DCN"
        greq.metadata_field.append("signature_def")
        gres = be.call("GetModelMetadata", greq, 10)
        sdm = pb.SignatureDefMap()
        assert gres.metadata["signature_def"].Unpack(sdm)
        sd = sdm.signature_def["serving_default"]
        assert sd.inputs["feat_ids"].dtype == pb.DT_INT64 and "prediction_node" in sd.outputs
        greq.metadata_field[0] = "bogus"
        with pytest.raises(grpc.RpcError):
            be.call("GetModelMetadata", greq, 10)
    finally:
        be.close()


def test_message_predict_and_batching(server):
    srv, _ = server
    svc = srv.service
    import concurrent.futures as cf

    reqs = [SyntheticRequestsMsg(i) for i in range(20)]
    with cf.ThreadPoolExecutor(8) as ex:
        resps = list(ex.map(svc.predict, reqs))
    for r, resp in zip(reqs, resps):
        got = T.to_ndarray(resp.outputs["prediction_node"])
        exp = _expected(srv, T.to_ndarray(r.inputs["feat_ids"]), T.to_ndarray(r.inputs["feat_wts"])).numpy()
        assert np.allclose(got, exp, atol=1e-6)
    st = srv.registry.resolve("DCN").scheduler.stats()
    assert st["batches"] >= 1 and st["rows_served"] >= 20


def SyntheticRequestsMsg(i):
    from distributed_tf_serving_amd.client.synth import SyntheticRequests

    return SyntheticRequests(dist="uniform", seed=i).message(1 + i % 5)


def test_oversized_request_is_split(server):
    srv, _ = server
    ids = torch.randint(0, 1000, (150, 43))  # > max_batch_rows (64): split into row chunks
    wts = torch.rand(150, 43)
    r = pb.PredictRequest()
    r.model_spec.name = "DCN"
    r.inputs["feat_ids"].CopyFrom(T.make_tensor_proto(ids.numpy()))
    r.inputs["feat_wts"].CopyFrom(T.make_tensor_proto(wts.numpy()))
    out = pb.PredictResponse.FromString(srv.service.predict_bytes(r.SerializeToString()))
    assert np.allclose(T.to_ndarray(out.outputs["prediction_node"]), _expected(srv, ids, wts).numpy(), atol=1e-6)


def test_service_error_codes():
    e = ServingError(Code.NOT_FOUND, "x")
    assert e.grpc_code() == grpc.StatusCode.NOT_FOUND


def test_prometheus_metrics(server):
    """TF-Serving's monitoring endpoint: RPC counts by API/status, latency
    histogram and the batching scheduler's counters, over HTTP."""
    import urllib.request

    srv, port = server
    be = GrpcBackend(f"127.0.0.1:{port}")
    try:
        be.predict(build_request(reference_shape=False).SerializeToString(), 30)
        bad = build_request(reference_shape=False)
        bad.model_spec.name = "nope"
        with pytest.raises(Exception):
            be.predict(bad.SerializeToString(), 30)
    finally:
        be.close()
    mport = srv.start_monitoring(0, "127.0.0.1")
    body = urllib.request.urlopen(f"http://127.0.0.1:{mport}/monitoring/prometheus/metrics", timeout=10).read()
    text = body.decode()
    assert ":tensorflow:serving:request_count_total" in text

    def val(prefix):
        lines = [ln for ln in text.splitlines() if ln.startswith(prefix)]
        assert lines, prefix
        return float(lines[0].rsplit(" ", 1)[1])

    assert val(':tensorflow:serving:request_count_total{API="Predict",status="OK"}') >= 1
    assert val(':tensorflow:serving:request_count_total{API="Predict",status="NOT_FOUND"}') >= 1
    assert val(':tensorflow:serving:request_latency_count{API="Predict"}') >= 2
    assert val(':tensorflow:serving:rows_served_total{model_name="DCN",version="1"}') >= 1
    assert val(':tensorflow:serving:batching_avg_batch_rows{model_name="DCN",version="1"}') > 0


def test_predict_ranked_outputs(server):
    """output_filter naming the ranked outputs: sorted_prediction ascending
    (the reference client's Collections.sort, DCNClient.java:195) and the
    candidate permutation it loses, over gRPC (bytes path) and in-process
    (message path); the live fast path routes such requests to the general
    path; unknown outputs stay INVALID_ARGUMENT."""
    srv, port = server
    rng = np.random.default_rng(3)
    ids = rng.integers(0, 1 << 40, (37, 43))
    wts = rng.random((37, 43), dtype=np.float32)
    req = pb.PredictRequest()
    req.model_spec.name = "DCN"
    req.inputs["feat_ids"].CopyFrom(T.make_tensor_proto(ids))
    req.inputs["feat_wts"].CopyFrom(T.make_tensor_proto(wts))
    want = _expected(srv, ids, wts).numpy()
    req.output_filter.extend(["prediction_node", "sorted_prediction", "sorted_index"])
    be = GrpcBackend(f"127.0.0.1:{port}")
    try:
        for resp in (pb.PredictResponse.FromString(be.predict(req.SerializeToString(), 30)),
                     srv.service.predict(req)):
            got = T.to_ndarray(resp.outputs["prediction_node"])
            srt = T.to_ndarray(resp.outputs["sorted_prediction"])
            perm = T.to_ndarray(resp.outputs["sorted_index"])
            assert np.allclose(got, want, atol=1e-6)
            assert perm.dtype == np.int64 and sorted(perm.tolist()) == list(range(37))
            assert np.all(np.diff(srt) >= 0) and np.array_equal(srt, got[perm])
        only = pb.PredictRequest()
        only.CopyFrom(req)
        del only.output_filter[:]
        only.output_filter.append("sorted_index")
        resp = pb.PredictResponse.FromString(be.predict(only.SerializeToString(), 30))
        assert list(resp.outputs.keys()) == ["sorted_index"]
        bad = pb.PredictRequest()
        bad.CopyFrom(req)
        bad.output_filter.append("nope")
        with pytest.raises(grpc.RpcError) as ei:
            be.predict(bad.SerializeToString(), 30)
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    finally:
        be.close()

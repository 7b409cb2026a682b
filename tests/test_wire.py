"""Wire layer: vendored schema, TensorProto codec (python + native), fill semantics."""
import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.packing import PackedLayout
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire import tensor as T


def reference_request(rows, F=43, raw=False):
    """Exactly what DCNClient.sendRequest builds (reference DCNClient.java:91-108)."""
    r = pb.PredictRequest()
    r.model_spec.name = "DCN"
    r.model_spec.signature_name = "serving_default"
    ids = np.tile(np.arange(1, F + 1, dtype=np.int64), rows).reshape(rows, F)
    r.inputs["feat_ids"].CopyFrom(T.make_tensor_proto(ids, raw=raw))
    r.inputs["feat_wts"].CopyFrom(T.make_tensor_proto(np.ones((rows, F), np.float32), raw=raw))
    return r


def test_schema_surface():
    assert set(pb.METHODS) == {"Classify", "Regress", "Predict", "MultiInference", "GetModelMetadata"}
    assert pb.SERVICE_NAME == "tensorflow.serving.PredictionService"
    assert pb.DT_INT64 == 9 and pb.DT_FLOAT == 1 and pb.DT_BFLOAT16 == 14


def test_reference_wire_sizes():
    # SURVEY.md §2.5 measured these with the reference's own protos
    assert len(reference_request(1500).SerializeToString()) == 322594
    assert len(reference_request(500).SerializeToString()) == 107594


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64, np.int8, np.uint8, np.int16,
                                   np.uint16, np.float16, np.bool_, np.uint32, np.uint64])
@pytest.mark.parametrize("raw", [False, True])
def test_tensor_roundtrip(dtype, raw):
    rng = np.random.default_rng(0)
    a = (rng.random((3, 5)) * 100).astype(dtype)
    tp = T.make_tensor_proto(a, raw=raw)
    tp2 = pb.TensorProto.FromString(tp.SerializeToString())
    b = T.to_ndarray(tp2)
    assert b.dtype == a.dtype and b.shape == a.shape
    assert np.array_equal(a, b)


def test_fill_semantics():
    tp = pb.TensorProto(dtype=pb.DT_INT64)
    tp.tensor_shape.CopyFrom(T.make_shape([2, 4]))
    tp.int64_val.extend([1, 2, 3])
    assert T.to_ndarray(tp).tolist() == [[1, 2, 3, 3], [3, 3, 3, 3]]
    empty = pb.TensorProto(dtype=pb.DT_FLOAT)
    empty.tensor_shape.CopyFrom(T.make_shape([3]))
    assert T.to_ndarray(empty).tolist() == [0, 0, 0]
    tp.int64_val.extend(range(10))
    with pytest.raises(T.InvalidArgument):
        T.to_ndarray(tp)
    bad = pb.TensorProto(dtype=pb.DT_FLOAT, tensor_content=b"\0" * 7)
    bad.tensor_shape.CopyFrom(T.make_shape([2]))
    with pytest.raises(T.InvalidArgument):
        T.to_ndarray(bad)


def test_bf16_tensor():
    t = torch.randn(4, 3).to(torch.bfloat16)
    for raw in (True, False):
        back = T.to_torch(pb.TensorProto.FromString(T.from_torch(t, raw=raw).SerializeToString()))
        assert back.dtype == torch.bfloat16 and torch.equal(back, t)


def test_native_parse_matches_python():
    nat = native()
    for raw in (False, True):
        msg = SyntheticRequests(dist="zipf", id_space=1 << 40, seed=3).message(37, raw=raw)
        msg.model_spec.version.value = 7
        msg.output_filter.append("prediction_node")
        b = msg.SerializeToString()
        p = nat.parse_predict_request(b)
        assert p.model_name == "DCN" and p.signature_name == "serving_default" and p.version == 7
        assert p.output_filter == ["prediction_node"]
        assert sorted(p.input_names()) == ["feat_ids", "feat_wts"]
        assert p.shape("feat_ids") == [37, 43] and p.dtype("feat_ids") == pb.DT_INT64
        ids = torch.empty(37 * 43, dtype=torch.int64)
        wts = torch.empty(37 * 43, dtype=torch.float32)
        p.decode_into("feat_ids", ids)
        p.decode_into("feat_wts", wts)
        assert np.array_equal(ids.view(37, 43).numpy(), T.to_ndarray(msg.inputs["feat_ids"]))
        assert np.array_equal(wts.view(37, 43).numpy(), T.to_ndarray(msg.inputs["feat_wts"]))
        # narrowing + hashing
        ids32 = torch.empty(37 * 43, dtype=torch.int32)
        p.decode_into("feat_ids", ids32, 0, 1000003)
        assert np.array_equal(ids32.numpy(), (T.to_ndarray(msg.inputs["feat_ids"]) % 1000003).reshape(-1))


def test_native_fill_and_errors():
    nat = native()
    # the reference smoke client: shape [1500,43] with 87 ids / 86 weights
    r = pb.PredictRequest()
    r.model_spec.name = "DCN"
    t = r.inputs["feat_ids"]
    t.dtype = pb.DT_INT64
    t.tensor_shape.CopyFrom(T.make_shape([1500, 43]))
    t.int64_val.extend(list(range(1, 44)) + list(range(43, 87)))
    w = r.inputs["feat_wts"]
    w.dtype = pb.DT_FLOAT
    w.tensor_shape.CopyFrom(T.make_shape([1500, 43]))
    w.float_val.extend([1.0] * 86)
    p = nat.parse_predict_request(r.SerializeToString())
    ids = torch.empty(1500 * 43, dtype=torch.int64)
    p.decode_into("feat_ids", ids)
    assert np.array_equal(ids.numpy(), T.to_ndarray(t).reshape(-1))
    assert ids[-1].item() == 86
    with pytest.raises(ValueError):
        nat.parse_predict_request(b"\x0a\xff\xff")
    too_many = pb.PredictRequest()
    tm = too_many.inputs["feat_ids"]
    tm.dtype = pb.DT_INT64
    tm.tensor_shape.CopyFrom(T.make_shape([1, 2]))
    tm.int64_val.extend([1, 2, 3])
    p = nat.parse_predict_request(too_many.SerializeToString())
    with pytest.raises(ValueError):
        p.decode_into("feat_ids", torch.empty(2, dtype=torch.int64))
    with pytest.raises(KeyError):
        p.decode_into("nope", torch.empty(2, dtype=torch.int64))


def test_native_encode_response_parses_in_python():
    nat = native()
    scores = torch.rand(500)
    for raw in (False, True):
        b = nat.encode_predict_response("DCN", "serving_default", 3, [("prediction_node", scores)], raw)
        r = pb.PredictResponse.FromString(b)
        assert r.model_spec.name == "DCN" and r.model_spec.version.value == 3
        out = T.to_ndarray(r.outputs["prediction_node"])
        assert np.array_equal(out, scores.numpy())
        if not raw:  # byte-identical to protobuf's own serializer for the float_val form
            assert r.SerializeToString() == b


def test_native_encode_request_roundtrip():
    nat = native()
    ids = torch.randint(0, 1 << 40, (9, 43))
    wts = torch.rand(9, 43)
    for raw in (False, True):
        b = nat.encode_predict_request("DCN", "serving_default", None, [("feat_ids", ids), ("feat_wts", wts)], raw,
                                       ["prediction_node"])
        r = pb.PredictRequest.FromString(b)
        assert not r.model_spec.HasField("version")
        assert list(r.output_filter) == ["prediction_node"]
        assert np.array_equal(T.to_ndarray(r.inputs["feat_ids"]), ids.numpy())
        assert np.array_equal(T.to_ndarray(r.inputs["feat_wts"]), wts.numpy())


@pytest.mark.parametrize("raw", [False, True])
def test_parse_batch_into_packed_rows(raw):
    nat = native()
    L = PackedLayout(43)
    synth = SyntheticRequests(dist="uniform", id_space=1 << 50, seed=1)
    msgs = [synth.message(n, raw=raw) for n in (5, 1, 300, 17)]
    bad = b"\x12\x03abc"  # truncated map entry
    reqs = [m.SerializeToString() for m in msgs[:2]] + [bad] + [m.SerializeToString() for m in msgs[2:]]
    batch = nat.parse_batch(reqs, "feat_ids", "feat_wts", 43)
    assert list(batch.rows) == [5, 1, 0, 300, 17]
    assert batch.errors[2] and not any(batch.errors[i] for i in (0, 1, 3, 4))
    buf = L.alloc(400)
    batch.decode(L.ids(buf), L.wts(buf))
    for i, m in zip((0, 1, 3, 4), msgs):
        o, n = batch.offsets[i], batch.rows[i]
        assert np.array_equal(L.ids(buf)[o:o + n].numpy(), T.to_ndarray(m.inputs["feat_ids"]))
        assert np.array_equal(L.wts(buf)[o:o + n].numpy(), T.to_ndarray(m.inputs["feat_wts"]))
    scores = torch.rand(batch.total_rows)
    outs = nat.encode_batch_responses("DCN", "serving_default", 1, "prediction_node", scores,
                                      list(batch.rows), list(batch.offsets))
    r3 = pb.PredictResponse.FromString(outs[3])
    o = batch.offsets[3]
    assert np.array_equal(T.to_ndarray(r3.outputs["prediction_node"]), scores[o:o + 300].numpy())


def test_parse_batch_shape_errors():
    nat = native()
    m = SyntheticRequests(fields=10, seed=0).message(4)
    b = nat.parse_batch([m.SerializeToString()], "feat_ids", "feat_wts", 43)
    assert b.rows[0] == 0 and "shape" in b.errors[0]
    b = nat.parse_batch([m.SerializeToString()], "missing", "feat_wts", 10)
    assert "missing" in b.errors[0]

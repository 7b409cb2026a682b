"""The native live server (csrc/runtime/live_server.cpp) on its CPU backend:
concurrent requests are batched into arenas, scored, answered per request;
validation, oversize split, deadlines, failure -> UNAVAILABLE, close, the native
load generator (closed and open loop) and lockstep stepping. Scores are
checked against the model's fp32 forward on the same rows."""
import concurrent.futures as cf
import threading

import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.errors import Code, ServingError
from distributed_tf_serving_amd.serving.live import LiveScheduler
from distributed_tf_serving_amd.serving.server import ModelServer, build_engine
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire import tensor as T

F = 43


def _cfg(max_rows=64, buckets=(8, 64), timeout_us=300):
    cfg = load_preset("wdl_tiny_cpu")
    cfg.serving.max_batch_rows = max_rows
    cfg.serving.allowed_batch_sizes = tuple(buckets)
    cfg.serving.batch_timeout_us = timeout_us
    return cfg


@pytest.fixture(scope="module")
def server():
    srv = ModelServer(_cfg(), device="cpu")
    yield srv
    srv.stop()


def _scores(resp: bytes) -> np.ndarray:
    return T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])


def _expected(srv, ids, wts):
    m = srv.registry.resolve("DCN").model
    return m(torch.as_tensor(ids), torch.as_tensor(wts)).numpy()


def test_server_uses_live_scheduler(server):
    s = server.registry.resolve("DCN")
    assert isinstance(s.scheduler, LiveScheduler)
    assert server.service._live_fast() is s.scheduler


@pytest.mark.parametrize("raw", [True, False])
def test_concurrent_requests_match_fp32_forward(server, raw):
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=3)
    reqs = []
    for i in range(48):
        rows = [1, 5, 17, 64, 3, 40][i % 6]
        ids, wts = synth.arrays(rows)
        data = native().encode_predict_request("DCN", "serving_default", None,
                                               [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                               raw)
        reqs.append((data, ids, wts))
    before = server.registry.resolve("DCN").scheduler.stats()["steps"]
    with cf.ThreadPoolExecutor(12) as pool:
        outs = list(pool.map(lambda r: server.service.predict_bytes(r[0], 10.0), reqs))
    for (data, ids, wts), resp in zip(reqs, outs):
        got = _scores(resp)
        assert got.shape == (ids.shape[0],)
        np.testing.assert_allclose(got, _expected(server, ids, wts), atol=1e-5)
    st = server.registry.resolve("DCN").scheduler.stats()
    assert st["steps"] > before
    # requests were coalesced: fewer steps than requests
    assert st["steps"] - before < len(reqs)


def test_packed_reference_request_with_fill_semantics(server):
    from distributed_tf_serving_amd.client.simple import build_request

    req = build_request(reference_shape=True)  # DCNClientSimple: [1500,43] with 87 ids -> oversize + fill
    resp = pb.PredictResponse.FromString(server.service.predict_bytes(req.SerializeToString(), 30.0))
    got = T.to_ndarray(resp.outputs["prediction_node"])
    ids = T.to_ndarray(req.inputs["feat_ids"])
    wts = T.to_ndarray(req.inputs["feat_wts"])
    assert got.shape == (1500,)  # 1500 rows > 64: split into batch-sized raw requests and joined
    np.testing.assert_allclose(got, _expected(server, ids, wts), atol=1e-5)


def test_validation_errors(server):
    live = server.registry.resolve("DCN").scheduler
    synth = SyntheticRequests(fields=F, seed=1)
    ok = synth.serialized(4)
    # wrong model name -> NOT_FOUND from the native server, same from the service
    other = SyntheticRequests(fields=F, seed=1, model_name="nope").serialized(4)
    code, msg, _ = live.predict_raw(other, 5.0)
    assert code == Code.NOT_FOUND
    with pytest.raises(ServingError) as ei:
        server.service.predict_bytes(other, 5.0)
    assert ei.value.code == Code.NOT_FOUND
    # wrong signature
    bad_sig = SyntheticRequests(fields=F, seed=1, signature_name="x").serialized(4)
    code, msg, _ = live.predict_raw(bad_sig, 5.0)
    assert code == Code.INVALID_ARGUMENT and "signature" in msg
    # wrong width
    bad_w = native().encode_predict_request("DCN", "", None, [("feat_ids", torch.zeros(2, 7, dtype=torch.int64)),
                                                              ("feat_wts", torch.zeros(2, 7))], True)
    code, msg, _ = live.predict_raw(bad_w, 5.0)
    assert code == Code.INVALID_ARGUMENT and "shape" in msg
    # garbage
    code, msg, _ = live.predict_raw(b"\x0a\x05garbage", 5.0)
    assert code == Code.INVALID_ARGUMENT
    # a good request still works afterwards
    code, msg, resp = live.predict_raw(ok, 5.0)
    assert code == 0 and _scores(resp).shape == (4,)


def test_overlong_varint_rejected_without_overwrite(server):
    """10+ continuation bytes must not turn into extra ids."""
    live = server.registry.resolve("DCN").scheduler

    def varint(v):
        out = bytearray()
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
        return bytes(out)

    ids = pb.TensorProto()
    ids.dtype = pb.DT_INT64
    ids.tensor_shape.dim.add().size = 1
    ids.tensor_shape.dim.add().size = F
    blob = bytes([0x80] * 20) + bytes([0x01]) + varint(5) * (F - 1)
    raw_ids = ids.SerializeToString() + bytes([0x52]) + varint(len(blob)) + blob  # field 10 (int64_val) packed
    req = pb.PredictRequest()
    req.model_spec.name = "DCN"
    req.inputs["feat_wts"].CopyFrom(T.make_tensor_proto(np.ones((1, F), np.float32)))
    data = bytearray(req.SerializeToString())
    key = b"feat_ids"
    entry = bytes([0x0A]) + varint(len(key)) + key + bytes([0x12]) + varint(len(raw_ids)) + raw_ids
    data += bytes([0x12]) + varint(len(entry)) + entry  # PredictRequest.inputs map entry
    data = bytes(data)
    # host decoder (slow path / parse_batch): rejected outright
    parsed = native().parse_predict_request(data)
    with pytest.raises(ValueError, match="10 bytes|more values"):
        parsed.decode_into("feat_ids", torch.zeros(1, F, dtype=torch.int64))
    # arena path (the GPU decodes varints: a value per terminator byte, at most
    # 10 bytes looked at): the request is answered with its declared shape and
    # a valid request batched right behind it is scored exactly
    synth = SyntheticRequests(fields=F, seed=11)
    ids, wts = synth.arrays(6)
    good = native().encode_predict_request("DCN", "", None,
                                           [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                           True)
    done = {}
    ev = threading.Event()

    def cb(name):
        def f(code, msg, resp):
            done[name] = (code, msg, resp)
            if len(done) == 2:
                ev.set()
        return f

    live.srv.submit(data, 5.0, cb("bad"))
    live.srv.submit(good, 5.0, cb("good"))
    assert ev.wait(10)
    code, msg, resp = done["bad"]
    assert code == Code.INVALID_ARGUMENT or _scores(resp).shape == (1,)
    code, msg, resp = done["good"]
    assert code == 0
    np.testing.assert_allclose(_scores(resp), _expected(server, ids, wts), atol=1e-5)


def test_max_request_rows_checked_before_allocation(server):
    live = server.registry.resolve("DCN").scheduler
    # a ~100-byte request declaring 10^8 rows (fill semantics) is refused up front
    ids = pb.TensorProto(dtype=pb.DT_INT64, int64_val=[1])
    ids.tensor_shape.dim.add().size = 100_000_000
    ids.tensor_shape.dim.add().size = F
    wts = pb.TensorProto(dtype=pb.DT_FLOAT, float_val=[1.0])
    wts.tensor_shape.CopyFrom(ids.tensor_shape)
    req = pb.PredictRequest()
    req.model_spec.name = "DCN"
    req.inputs["feat_ids"].CopyFrom(ids)
    req.inputs["feat_wts"].CopyFrom(wts)
    with pytest.raises(ServingError) as ei:
        server.service.predict_bytes(req.SerializeToString(), 5.0)
    assert ei.value.code == Code.INVALID_ARGUMENT and "at most" in ei.value.message
    assert live.max_request_rows < 100_000_000


def test_classify_and_predict_messages_use_live_engine(server):
    synth = SyntheticRequests(fields=F, seed=9)
    msg = synth.message(70)  # > one 64-row batch: two raw sub-requests
    resp = server.service.predict(msg, 10.0)
    ids = T.to_ndarray(msg.inputs["feat_ids"])
    wts = T.to_ndarray(msg.inputs["feat_wts"])
    np.testing.assert_allclose(T.to_ndarray(resp.outputs["prediction_node"]), _expected(server, ids, wts), atol=1e-5)


def test_native_load_generator_closed_and_open_loop(server):
    live = server.registry.resolve("DCN").scheduler
    synth = SyntheticRequests(fields=F, seed=5)
    reqs = [synth.serialized(16) for _ in range(8)]
    r = live.run_load(reqs, warmup=8, count=64, concurrency=8, threads=3)
    assert r["ok"] == r["submitted"] == 8 + 64 + 8 and r["errors"] == 0
    assert len(r["latency_us"]) == 64 and r["window_us"] > 0
    r = live.run_load(reqs, warmup=4, count=40, qps=2000.0, threads=2)
    assert r["ok"] == 44 and len(r["latency_us"]) == 40
    assert all(x > 0 for x in r["latency_us"])


def _engine(cfg):
    return build_engine(cfg, device="cpu", slots=2)


def test_deadline_and_close_and_broken():
    cfg = _cfg(max_rows=8, buckets=(8,), timeout_us=100)
    eng = _engine(cfg)
    live = LiveScheduler(eng, cfg.serving)
    synth = SyntheticRequests(fields=F, seed=2)
    data = synth.serialized(8)
    assert live.predict_raw(data, 5.0)[0] == 0
    live.close()
    code, msg, _ = live.predict_raw(data, 5.0)
    assert code == Code.UNAVAILABLE
    # a forward that fails marks the server broken: every later request UNAVAILABLE, no hang
    eng2 = _engine(cfg)
    calls = {"n": 0}
    orig = eng2.launch

    def bad_launch(*a, **k):
        calls["n"] += 1
        if calls["n"] >= 2:
            raise RuntimeError("injected device failure")
        return orig(*a, **k)

    eng2.launch = bad_launch
    live2 = LiveScheduler(eng2, cfg.serving)
    assert live2.predict_raw(data, 5.0)[0] == 0
    code, msg, _ = live2.predict_raw(data, 5.0)
    assert code == Code.UNAVAILABLE and "injected" in msg
    assert live2.broken
    assert live2.predict_raw(data, 5.0)[0] == Code.UNAVAILABLE
    live2.close()


def test_cluster_mode_steps_only_on_demand_at_the_smallest_bucket():
    """A live server with a step control (one rank): no step while idle, a
    lone small request runs the small bucket, not the largest."""
    import os

    from distributed_tf_serving_amd.parallel.control import create_control

    cfg = _cfg(max_rows=8, buckets=(4, 8), timeout_us=200)
    eng = _engine(cfg)
    store = torch.distributed.HashStore()
    ctl = create_control(native(), 1, 0, store=store, prefix=f"t/{os.getpid()}")
    live = LiveScheduler(eng, cfg.serving, control=ctl)
    threading.Event().wait(0.2)
    assert live.stats()["steps"] == 0  # idle: nothing launched
    synth = SyntheticRequests(fields=F, seed=4)
    for rows in (3, 7, 2):
        code, _, resp = live.predict_raw(synth.serialized(rows), 5.0)
        assert code == 0 and _scores(resp).shape == (rows,)
    threading.Event().wait(0.2)
    st = live.stats()
    assert st["steps"] == 3 and st["empty_steps"] == 0 and st["proposed_steps"] == 3
    assert st["padded_rows"] == 4 + 8 + 4  # each step sized to its batch
    assert ctl.proposed == 3
    live.close()
    assert ctl.all_closing


def test_host_narrowing_matches_python():
    """runtime/narrow.cpp (AVX2 + scalar tails) vs python's modulo."""
    rng = np.random.default_rng(0)
    vals = np.concatenate([rng.integers(0, 1 << 40, 4099), rng.integers(-(1 << 62), 1 << 62, 1001),
                           np.array([0, 1, -1, (1 << 52) - 1, 1 << 52, (1 << 63) - 1, -(1 << 63), 999_999,
                                     1_000_000, 2_000_000, -1_000_000], dtype=np.int64)]).astype(np.int64)
    for m in (1, 7, 1_000_000, (1 << 31) - 1):
        got = native().narrow_ids(torch.from_numpy(vals), m).numpy()
        want = np.array([int(v) % m for v in vals.tolist()], dtype=np.int64)
        assert np.array_equal(got.astype(np.int64), want), m


def test_host_narrowing_to_3_byte_rows_matches_python():
    """runtime/narrow.cpp narrow_ids24 (AVX2 shuffle pack + scalar tail) vs
    python's modulo, every length mod 8 and across the 2048-id blocks."""
    rng = np.random.default_rng(5)
    for n in (1, 7, 8, 9, 2047, 2048, 2049, 5003):
        vals = rng.integers(-(1 << 62), 1 << 62, size=n, dtype=np.int64)
        for m in (1, 1_000_000, 1 << 24):
            got = native().narrow_ids24(torch.from_numpy(vals), m).numpy().reshape(n, 3).astype(np.int64)
            rows = got[:, 0] | (got[:, 1] << 8) | (got[:, 2] << 16)
            want = np.array([int(v) % m for v in vals.tolist()], dtype=np.int64)
            assert np.array_equal(rows, want), (n, m)


def test_live_server_narrowed_ingest_matches_fp32_forward_for_every_encoding():
    """Host-narrowed rows (int32 table rows + fp32 weights) and packed varint
    requests score exactly like the fp32 forward: the wire encoding does not
    change a request's scores."""
    cfg = _cfg(max_rows=64, buckets=(8, 64))
    cfg.model.vocab_size = 100_000
    eng = _engine(cfg)
    live = LiveScheduler(eng, cfg.serving, narrow=True)
    assert live.narrow_modulo == 100_000
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=12)
    model = eng.ex.model
    reqs = []
    for rows in (1, 9, 33, 64, 5):
        ids, wts = synth.arrays(rows)
        raw = native().encode_predict_request("DCN", "", None, [("feat_ids", torch.from_numpy(ids)),
                                                                ("feat_wts", torch.from_numpy(wts))], True)
        packed = native().encode_predict_request("DCN", "", None, [("feat_ids", torch.from_numpy(ids)),
                                                                   ("feat_wts", torch.from_numpy(wts))], False)
        reqs.append((raw, packed, ids, wts))
    with cf.ThreadPoolExecutor(6) as pool:
        outs = list(pool.map(lambda r: (live.predict_bytes(r[0], 10.0), live.predict_bytes(r[1], 10.0)), reqs))
    for (raw, packed, ids, wts), (r_raw, r_packed) in zip(reqs, outs):
        want32 = model(torch.from_numpy(ids), torch.from_numpy(wts)).numpy()
        np.testing.assert_allclose(_scores(r_raw), want32, atol=1e-5)      # narrowed ids, fp32 weights
        np.testing.assert_allclose(_scores(r_packed), want32, atol=1e-5)   # packed varint ids travel raw
    assert live.stats()["narrowed"] == len(reqs)
    live.close()


def test_live_server_narrowed_weights_travel_in_their_cheapest_exact_form():
    """Host narrowing picks each request's weight form: all 1.0 (the reference
    client's requests, DCNClient.java:67-73) -> no weight bytes at all, every
    weight exactly a bf16 value -> bf16, else fp32. Mixed in one batch, every
    request scores exactly like the fp32 forward of its own weights, and the
    arena carries fewer bytes for the cheaper forms."""
    cfg = _cfg(max_rows=64, buckets=(8, 64))
    cfg.model.vocab_size = 100_000
    eng = _engine(cfg)
    live = LiveScheduler(eng, cfg.serving, narrow=True)
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=21)
    model = eng.ex.model
    reqs = []
    for rows, kind in ((5, "ones"), (17, "bf16"), (9, "f32"), (30, "ones"), (3, "bf16")):
        ids, wts = synth.arrays(rows)
        if kind == "ones":
            wts = np.ones_like(wts)
        elif kind == "bf16":
            wts = torch.from_numpy(wts).to(torch.bfloat16).float().numpy()
        t = [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(np.ascontiguousarray(wts)))]
        reqs.append((native().encode_predict_request("DCN", "", None, t, True), ids, wts))
    with cf.ThreadPoolExecutor(5) as pool:
        outs = list(pool.map(lambda r: live.predict_bytes(r[0], 10.0), reqs))
    for (raw, ids, wts), out in zip(reqs, outs):
        want = model(torch.from_numpy(ids), torch.from_numpy(wts)).numpy()
        np.testing.assert_allclose(_scores(out), want, atol=1e-5)
    st = live.stats()
    assert st["narrowed"] == 5 and st["narrowed_wts_implicit"] == 2 and st["narrowed_wts_bf16"] == 2, st
    live.close()


def test_weight_kind_classification():
    """runtime/narrow.cpp classify_weights: all 1.0 -> 2 (implicit), all exact
    bf16 -> 1, else 0 - over the columns the model reads only."""
    vals = np.array([[1.0, 1.0, 1.0], [0.5, -2.0, 0.375]], dtype=np.float32)
    assert native().classify_weights(torch.from_numpy(np.ones((4, 3), np.float32)), 3) == 2
    assert native().classify_weights(torch.from_numpy(vals[1:].copy()), 3) == 1
    assert native().classify_weights(torch.from_numpy(np.full((2, 3), 0.1, np.float32)), 3) == 0
    # only the columns the model reads decide: a non-bf16 value beyond wcols does not matter
    mixed = np.array([[1.0, 1.0, 0.1]], dtype=np.float32)
    assert native().classify_weights(torch.from_numpy(mixed), 2) == 2 and native().classify_weights(
        torch.from_numpy(mixed), 3) == 0


def test_live_server_narrow_weight_columns_for_one_hot_dlrm():
    """One-hot DLRM reads only its 13 dense weights: host-narrowed requests
    carry just those (the arena header tells the readers), and the served
    scores still equal the fp32 forward of the full request, raw and packed
    encodings alike."""
    from distributed_tf_serving_amd.config import ModelConfig

    cfg = _cfg(max_rows=64, buckets=(8, 64))
    cfg.model = ModelConfig(family="dlrm", table_rows=5000, param_dtype="fp32")
    eng = _engine(cfg)
    live = LiveScheduler(eng, cfg.serving, narrow=True)
    assert live.narrow_modulo == 5000 and live.narrow_wts_cols == 13
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=13)
    model = eng.ex.model
    reqs = []
    for rows in (1, 7, 33, 64):
        ids, wts = synth.arrays(rows)
        t = [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))]
        reqs.append((native().encode_predict_request("DCN", "", None, t, True),
                     native().encode_predict_request("DCN", "", None, t, False), ids, wts))
    with cf.ThreadPoolExecutor(4) as pool:
        outs = list(pool.map(lambda r: (live.predict_bytes(r[0], 10.0), live.predict_bytes(r[1], 10.0)), reqs))
    for (raw, packed, ids, wts), (r_raw, r_packed) in zip(reqs, outs):
        want = model(torch.from_numpy(ids), torch.from_numpy(wts)).numpy()
        np.testing.assert_allclose(_scores(r_raw), want, atol=1e-5)
        np.testing.assert_allclose(_scores(r_packed), want, atol=1e-5)
    assert live.stats()["narrowed"] == len(reqs)
    live.close()


def test_load_generator_waits_for_the_last_completion_callback(server):
    """Regression (round 3): run_load returned as soon as the last completion
    was counted, while that callback still went on to touch run_load's stack
    (next / work) on the completer thread - a use-after-return that surfaced as
    an intermittent SIGSEGV. The hook holds the final callback 150 ms after it
    counts; run_load must not return before the callback is done."""
    live = server.registry.resolve("DCN").scheduler
    synth = SyntheticRequests(fields=F, seed=6)
    reqs = [synth.serialized(16) for _ in range(4)]
    for kw in (dict(concurrency=4, threads=2), dict(qps=3000.0, threads=2)):
        r = live.run_load(reqs, warmup=2, count=12, debug_done_delay_us=150_000, **kw)
        assert r["errors"] == 0 and r["ok"] == r["submitted"]
        assert r["wall_us"] >= 150_000, r["wall_us"]

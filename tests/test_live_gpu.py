"""The native live server on the GPU backend (StepRunner + captured step
kernels): concurrent served requests vs the model's eager forward, bucket
choice for partial batches, the native load generator, bounded waits."""
import concurrent.futures as cf

import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import load_preset
from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.errors import Code
from distributed_tf_serving_amd.serving.live import LiveScheduler
from distributed_tf_serving_amd.serving.server import ModelServer
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire import tensor as T

pytestmark = pytest.mark.gpu
F = 43


@pytest.fixture(scope="module")
def server():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cfg = load_preset("deepfm_1gpu")
    cfg.model.vocab_size = 200_000
    cfg.serving.max_batch_rows = 2048
    cfg.serving.allowed_batch_sizes = (256, 2048)
    srv = ModelServer(cfg, device="cuda:0")
    yield srv
    srv.stop()


def _scores(resp):
    return T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])


def test_gpu_server_is_live(server):
    s = server.registry.resolve("DCN")
    assert isinstance(s.scheduler, LiveScheduler)
    assert type(s.scheduler.srv).__module__.endswith("_hip")


@pytest.mark.parametrize("raw", [True, False])
def test_concurrent_served_requests_match_eager_forward(server, raw):
    model = server.registry.resolve("DCN").model
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=21)
    reqs = []
    for i in range(40):
        rows = [512, 1, 100, 37, 300][i % 5]
        ids, wts = synth.arrays(rows)
        data = native().encode_predict_request("DCN", "serving_default", None,
                                               [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                               raw)
        reqs.append((data, ids, wts))
    with cf.ThreadPoolExecutor(16) as pool:
        outs = list(pool.map(lambda r: server.service.predict_bytes(r[0], 30.0), reqs))
    live = server.registry.resolve("DCN").scheduler
    for (data, ids, wts), resp in zip(reqs, outs):
        got = _scores(resp)
        w = torch.from_numpy(wts).cuda()  # every encoding keeps fp32 weights
        want = model(torch.from_numpy(ids).cuda(), w).float().cpu().numpy()
        np.testing.assert_allclose(got, want, atol=2e-5)
    st = live.stats()
    assert st["steps"] < st["submitted"] and not st["broken"]
    if raw:
        assert st["narrowed"] > 0


def test_oversize_request_split(server):
    model = server.registry.resolve("DCN").model
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="uniform", seed=5)
    ids, wts = synth.arrays(5000)  # > 2048 rows: three batch-sized parts
    data = native().encode_predict_request("DCN", "", None, [("feat_ids", torch.from_numpy(ids)),
                                                             ("feat_wts", torch.from_numpy(wts))], True)
    got = _scores(server.service.predict_bytes(data, 30.0))
    w = torch.from_numpy(wts).cuda()  # split parts travel raw -> narrowed ids, fp32 weights
    want = model(torch.from_numpy(ids).cuda(), w).float().cpu().numpy()
    np.testing.assert_allclose(got, want, atol=2e-5)


def test_native_load_generator(server):
    live = server.registry.resolve("DCN").scheduler
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=8)
    reqs = [synth.serialized(512) for _ in range(16)]
    r = live.run_load(reqs, warmup=32, count=256, concurrency=32, threads=4, timeout_us=20_000_000)
    assert r["errors"] == 0 and r["ok"] == r["submitted"] and len(r["latency_us"]) == 256
    q = live.run_load(reqs, warmup=20, count=200, qps=4000.0, threads=2, timeout_us=20_000_000)
    assert q["errors"] == 0 and len(q["latency_us"]) == 200
    assert np.median(q["latency_us"]) < 20_000  # us


def test_deadline_exceeded_reported(server):
    live = server.registry.resolve("DCN").scheduler
    synth = SyntheticRequests(fields=F, seed=1)
    code, msg, _ = live.predict_raw(synth.serialized(64), 1e-6)
    assert code in (0, Code.DEADLINE_EXCEEDED)


def test_ranked_outputs_use_gpu_sort(server):
    """A request naming the ranked outputs leaves the live fast path and is
    served with the K7 bitonic sort on the GPU: sorted scores ascending and
    the candidate permutation, consistent with prediction_node."""
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=8)
    ids, wts = synth.arrays(1500)  # the reference request size
    data = native().encode_predict_request("DCN", "serving_default", None,
                                           [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                           True, ["prediction_node", "sorted_prediction", "sorted_index"])
    resp = pb.PredictResponse.FromString(server.service.predict_bytes(data, 30.0))
    got = T.to_ndarray(resp.outputs["prediction_node"])
    srt = T.to_ndarray(resp.outputs["sorted_prediction"])
    perm = T.to_ndarray(resp.outputs["sorted_index"])
    assert got.shape == (1500,) and sorted(perm.tolist()) == list(range(1500))
    assert np.all(np.diff(srt) >= 0) and np.array_equal(srt, got[perm])


def test_gather_gemm_served_steps_match_eager_forward():
    """Served steps at a bucket that takes the gather-GEMM path (K1 inside the
    first layer's GEMM, reading host-narrowed and raw arena rows): every
    request's scores match the model's eager forward."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_tf_serving_amd import ops

    cfg = load_preset("deepfm_1gpu")
    cfg.model.vocab_size = 200_000
    cfg.serving.max_batch_rows = max(8192, ops.GATHER_GEMM_MIN_ROWS)
    cfg.serving.allowed_batch_sizes = (cfg.serving.max_batch_rows,)
    srv = ModelServer(cfg, device="cuda:0")
    try:
        model = srv.registry.resolve("DCN").model
        assert model._gather_gemm(torch.zeros(cfg.serving.max_batch_rows, F, dtype=torch.int64, device="cuda"),
                                  None, fm2=True)
        synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=33)
        reqs = []
        for i in range(24):
            ids, wts = synth.arrays([512, 3, 700, 129][i % 4])
            data = native().encode_predict_request("DCN", "serving_default", None,
                                                   [("feat_ids", torch.from_numpy(ids)),
                                                    ("feat_wts", torch.from_numpy(wts))], i % 3 != 2)
            reqs.append((data, ids, wts))
        with cf.ThreadPoolExecutor(16) as pool:
            outs = list(pool.map(lambda r: srv.service.predict_bytes(r[0], 30.0), reqs))
        for (data, ids, wts), resp in zip(reqs, outs):
            want = model(torch.from_numpy(ids).cuda(), torch.from_numpy(wts).cuda()).float().cpu().numpy()
            np.testing.assert_allclose(_scores(resp), want, atol=5e-5)
        st = srv.registry.resolve("DCN").scheduler.stats()
        assert st["narrowed"] > 0 and not st["broken"]
    finally:
        srv.stop()


@pytest.mark.parametrize("kind", ["ones", "bf16", "mixed"])
def test_served_weight_kinds_match_eager_forward(server, kind):
    """Host narrowing ships all-1.0 weights as nothing and bf16-exact weights
    as bf16 (the GPU readers widen them back, csrc/kernels/common.h
    arena_narrow_w): scores equal the eager forward of the request's fp32
    weights, including a 2048-row gather-GEMM batch mixing every kind."""
    model = server.registry.resolve("DCN").model
    live = server.registry.resolve("DCN").scheduler
    st0 = live.stats()
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=31)
    reqs = []
    for i in range(12):
        ids, wts = synth.arrays([512, 1, 100, 37, 300, 512][i % 6])
        k = kind if kind != "mixed" else ["ones", "bf16", "f32"][i % 3]
        if k == "ones":
            wts = np.ones_like(wts)
        elif k == "bf16":
            wts = torch.from_numpy(wts).to(torch.bfloat16).float().numpy()
        t = [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(np.ascontiguousarray(wts)))]
        reqs.append((native().encode_predict_request("DCN", "serving_default", None, t, True), ids, wts))
    with cf.ThreadPoolExecutor(12) as pool:
        outs = list(pool.map(lambda r: server.service.predict_bytes(r[0], 30.0), reqs))
    for (data, ids, wts), resp in zip(reqs, outs):
        want = model(torch.from_numpy(ids).cuda(), torch.from_numpy(wts).cuda()).float().cpu().numpy()
        np.testing.assert_allclose(_scores(resp), want, atol=2e-5)
    st = live.stats()
    if kind in ("ones", "mixed"):
        assert st["narrowed_wts_implicit"] > st0["narrowed_wts_implicit"]
    if kind in ("bf16", "mixed"):
        assert st["narrowed_wts_bf16"] > st0["narrowed_wts_bf16"]


def test_one_hot_dlrm_served_from_narrow_arena_matches_eager():
    """One-hot DLRM on the GPU live server: host-narrowed requests carry only
    the 13 dense weights, the fused bottom MLP and the fused gather +
    interaction read the arena directly, and the scores equal the eager
    forward of the full request (raw and packed encodings)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_tf_serving_amd.config import ModelConfig

    cfg = load_preset("deepfm_1gpu")
    cfg.model = ModelConfig(family="dlrm", table_rows=20_000)
    cfg.serving.max_batch_rows = 2048
    cfg.serving.allowed_batch_sizes = (256, 2048)
    srv = ModelServer(cfg, device="cuda:0")
    try:
        s = srv.registry.resolve("DCN")
        live, model = s.scheduler, s.model
        assert isinstance(live, LiveScheduler) and model.supports_arena
        assert live.narrow_wts_cols == 13
        synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=23)
        reqs = []
        for i in range(20):
            ids, wts = synth.arrays([512, 1, 100, 37, 300][i % 5])
            t = [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))]
            reqs.append((native().encode_predict_request("DCN", "serving_default", None, t, i % 2 == 0), ids, wts))
        with cf.ThreadPoolExecutor(8) as pool:
            outs = list(pool.map(lambda r: srv.service.predict_bytes(r[0], 30.0), reqs))
        for (data, ids, wts), resp in zip(reqs, outs):
            want = model(torch.from_numpy(ids).cuda(), torch.from_numpy(wts).cuda()).float().cpu().numpy()
            np.testing.assert_allclose(_scores(resp), want, atol=2e-5)
        st = live.stats()
        assert st["narrowed"] > 0 and not st["broken"]
    finally:
        srv.stop()


def test_numa_placement_and_node_local_pinned_arena():
    """utils/affinity.py on the GPU box: the GPU's PCI bus id resolves, and a
    node-local arena is pinned (hipHostRegister) with its pages on the node;
    an H2D copy from it is exact."""
    from distributed_tf_serving_amd.ops import hip
    from distributed_tf_serving_amd.utils import affinity

    bus = hip().pci_bus_id(0)
    assert bus.count(":") == 2, bus
    node = native().pci_numa_node(bus)
    t = hip().alloc_pinned_on_node(4 << 20, max(node, 0))
    assert t.is_pinned()
    t[:] = torch.arange(4 << 20, dtype=torch.int64).remainder(251).to(torch.uint8)
    d = t.to("cuda:0", non_blocking=True)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), t)
    pg = native().page_numa_node(t, 0)
    if pg >= 0:
        assert pg == max(node, 0)
    a = affinity.alloc_pinned_arena(1 << 20)
    assert a.is_pinned() and a.numel() == 1 << 20


def test_native_grpc_front_door_on_gpu(server):
    """The native h2c front door over the GPU live server (csrc/net/h2_server.cpp
    calling the _hip module's LiveServer::submit), driven by the native client."""
    from distributed_tf_serving_amd.serving.native_front import NativeGrpcFront

    live = server.registry.resolve("DCN").scheduler
    fr = NativeGrpcFront(server.service, live, port=0, host="127.0.0.1", threads=2)
    try:
        synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=21)
        ids, wts = synth.arrays(300)
        data = native().encode_predict_request("DCN", "serving_default", None,
                                               [("feat_ids", torch.from_numpy(ids)), ("feat_wts", torch.from_numpy(wts))],
                                               True)
        st, msg, body = native().grpc_call("127.0.0.1", fr.port, "/tensorflow.serving.PredictionService/Predict",
                                           data, 30.0)
        assert st == 0, msg
        m = server.registry.resolve("DCN").model
        want = m(torch.from_numpy(ids).cuda(), torch.from_numpy(wts).cuda()).float().cpu().numpy()
        np.testing.assert_allclose(_scores(body), want, atol=2e-3)
        r = native().run_grpc_load("127.0.0.1", fr.port, "/tensorflow.serving.PredictionService/Predict",
                                   [data], concurrency=6, warmup=12, count=120, timeout_s=30.0)
        assert r["errors"] == 0 and r["ok"] == 132, r["first_error"]
    finally:
        fr.stop()

"""Failure paths (SURVEY.md §4 "Fault tests", §5.3): a failing or stalled shard
makes the request fail within its deadline (never hang), fail-over re-splits
the shard over the surviving backends, malformed input is INVALID_ARGUMENT."""
import time

import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.client.backends import InProcessBackend
from distributed_tf_serving_amd.client.fanout_client import FanoutClient, RequestSpec, ShardError
from distributed_tf_serving_amd.config import Config, ModelConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.serving.errors import Code, ServingError
from distributed_tf_serving_amd.serving.faults import FaultInjector, FaultSpec, FaultyBackend, FaultyService
from distributed_tf_serving_amd.serving.server import ModelServer


@pytest.fixture(scope="module")
def server():
    cfg = Config()
    cfg.model = ModelConfig(family="deepfm", vocab_size=5000, embed_dim=16, mlp_dims=(32, 16))
    cfg.serving.device = "cpu"
    cfg.serving.max_batch_rows = 256
    cfg.serving.allowed_batch_sizes = (64, 256)
    srv = ModelServer(cfg, device="cpu")
    yield srv, build_model(cfg.model)
    srv.stop()


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    return (torch.from_numpy(rng.integers(0, 1 << 40, size=(n, 43), dtype=np.int64)),
            torch.from_numpy(rng.random((n, 43), dtype=np.float32)))


def test_fault_spec_parse():
    f = FaultSpec.parse("after:5,kind:delay,ms:20,every:2")
    assert (f.after, f.kind, f.ms, f.every) == (5, "delay", 20.0, 2)
    with pytest.raises(ValueError):
        FaultSpec.parse("kind:explode")
    with pytest.raises(ValueError):
        FaultSpec.parse("bogus:1")


def test_injector_error_after_n():
    inj = FaultInjector(FaultSpec.parse("after:2,kind:error"))
    inj.check()
    inj.check()
    with pytest.raises(ServingError) as e:
        inj.check()
    assert e.value.code == Code.UNAVAILABLE and inj.injected == 1


def test_shard_failure_surfaces_with_shard_index(server):
    srv, _ = server
    good = InProcessBackend(srv.service, "good")
    bad = FaultyBackend(InProcessBackend(srv.service, "bad"), FaultInjector(FaultSpec.parse("after:0,kind:error")))
    cli = FanoutClient([good, bad], RequestSpec(model_name="DCN"), pool_threads=4)
    ids, wts = _data(20)
    with pytest.raises(ShardError) as e:
        cli.predict(ids, wts)
    assert e.value.shard == 1
    cli.pool.shutdown()


def test_failover_resplits_over_survivors(server):
    srv, ref = server
    backs = [InProcessBackend(srv.service, f"b{i}") for i in range(3)]
    backs[1] = FaultyBackend(backs[1], FaultInjector(FaultSpec.parse("after:0,kind:error")))
    cli = FanoutClient(backs, RequestSpec(model_name="DCN"), pool_threads=6, failover=True, cooldown_s=60)
    ids, wts = _data(31, seed=1)
    res = cli.predict(ids, wts)
    want = ref(ids, wts)
    assert torch.allclose(res.scores, want, atol=1e-5)  # candidate order preserved
    assert cli.failovers == 1
    assert cli.healthy() == [0, 2]
    res2 = cli.predict(ids, wts)  # new requests skip the backend in cool-down
    assert torch.allclose(res2.scores, want, atol=1e-5) and cli.failovers == 1
    cli.pool.shutdown()


def test_hung_shard_fails_within_deadline(server):
    srv, _ = server
    inj = FaultInjector(FaultSpec.parse("after:0,kind:hang"))
    hung = FaultyBackend(InProcessBackend(srv.service, "hung"), inj)
    cli = FanoutClient([InProcessBackend(srv.service), hung], RequestSpec(model_name="DCN"), pool_threads=4,
                       timeout_s=0.3)
    ids, wts = _data(10, seed=2)
    t0 = time.monotonic()
    with pytest.raises(ShardError) as e:
        cli.predict(ids, wts)
    assert time.monotonic() - t0 < 5.0
    assert isinstance(e.value.cause, ServingError) and e.value.cause.code == Code.DEADLINE_EXCEEDED
    inj.release()
    cli.pool.shutdown()


def test_faulty_service_wrapper(server):
    srv, _ = server
    svc = FaultyService(srv.service, FaultInjector(FaultSpec.parse("after:1,kind:error")))
    cli = FanoutClient([InProcessBackend(svc)], RequestSpec(model_name="DCN"), pool_threads=2)
    ids, wts = _data(5, seed=3)
    cli.predict(ids, wts)  # first request passes
    with pytest.raises(ShardError):
        cli.predict(ids, wts)
    assert svc.get_model_metadata is not None  # other RPCs pass through
    cli.pool.shutdown()


def test_malformed_request_is_invalid_argument(server):
    srv, _ = server
    with pytest.raises(ServingError) as e:
        srv.service.predict_bytes(b"\x0a\x05garbage-not-a-request", 5.0)
    assert e.value.code == Code.INVALID_ARGUMENT

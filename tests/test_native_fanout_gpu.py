"""Native RCCL communicators (csrc/comm) and the C++ fan-out step
(StepRunner.launch_fanout) on one GPU: a 1-rank communicator runs the same
all-to-all / scatter-gather code as an 8-rank one, so the whole N > 1 step
(H2D -> ingress graph -> collective -> forward graph -> collective -> D2H on
four streams) is exercised and checked against a local forward."""
import pytest
import torch

from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.parallel.dist import DistContext
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine
from distributed_tf_serving_amd.serving.arena import ArenaLayout
from distributed_tf_serving_amd.serving.executor import ShardExecutor
from distributed_tf_serving_amd.serving.packing import PackedLayout

pytestmark = pytest.mark.gpu


def test_rccl_comm_single_rank(cuda):
    from distributed_tf_serving_amd.parallel.native_comm import create_comm

    c = create_comm(DistContext(device=cuda))
    assert c.nranks == 1 and c.rank == 0
    x = torch.arange(1000, dtype=torch.float32, device=cuda)
    y = torch.zeros_like(x)
    c.alltoall(x, y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    z = torch.zeros_like(x)
    c.allgather(x, z)
    torch.cuda.synchronize()
    assert torch.equal(x, z)
    assert c.async_error() == ""
    c.abort()
    assert c.aborted


@pytest.mark.parametrize("mode,raw", [("local", True), ("local", False), ("alltoall", True), ("alltoall", False),
                                      ("scatter", True)])
def test_live_server_every_step_kind(cuda, mode, raw):
    """The GPU live server (parse -> H2D + step kernels / fan-out step ->
    encode) on one rank for each step kind - local direct launches, the native
    fan-out step (RCCL all-to-all / scatter+gather with the rank itself) - with
    raw and packed-varint requests (the latter decoded on the GPU): every
    request's scores match a local forward."""
    import concurrent.futures as cf

    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.config import ServingConfig
    from distributed_tf_serving_amd.ops import native
    from distributed_tf_serving_amd.serving.live import LiveScheduler
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    cfg = ModelConfig(family="deepfm", vocab_size=50_000)
    m = build_model(cfg, cuda)
    F = cfg.num_fields
    B, S = 1024, 4
    narrow = mode != "local"
    L = PackedLayout(F, cfg.vocab_size if narrow else 0)
    ex = ShardExecutor(m, L, [256, B], cuda, slots=S)
    AL = ArenaLayout(F, max_rows=B)
    eng = FanoutEngine(ex, DistContext(device=cuda), mode="alltoall" if mode == "local" else mode, ingest="arena",
                       arena=AL, force_fanout=mode != "local")
    for b in (256, B):
        eng.prepare(b)
    assert eng.native_fanout_active == (mode != "local")
    sc = ServingConfig(max_batch_rows=B, allowed_batch_sizes=(256, B), batch_timeout_us=300)
    live = LiveScheduler(eng, sc, depth=S - 1, step_timeout_s=20)
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=5)
    reqs = []
    for i in range(24):
        ids, wts = synth.arrays([1, 200, 37, 512][i % 4])
        reqs.append((native().encode_predict_request("DCN", "serving_default", None,
                                                     [("feat_ids", torch.from_numpy(ids)),
                                                      ("feat_wts", torch.from_numpy(wts))], raw), ids, wts))
    with cf.ThreadPoolExecutor(8) as pool:
        outs = list(pool.map(lambda r: live.predict_bytes(r[0], 30.0), reqs))
    for (data, ids, wts), resp in zip(reqs, outs):
        got = T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])
        want = m(torch.from_numpy(ids).to(cuda), torch.from_numpy(wts).to(cuda)).float().cpu().numpy()
        assert abs(got - want).max() < 2e-5
    st = live.stats()
    assert st["steps"] < len(reqs) and not st["broken"]
    live.close()


@pytest.mark.parametrize("mode", ["alltoall", "scatter"])
@pytest.mark.parametrize("ingest", ["packed", "arena", "arena-narrow"])
def test_native_fanout_step_matches_local(cuda, mode, ingest):
    cfg = ModelConfig(family="deepfm", vocab_size=50_000)
    m = build_model(cfg, cuda)
    narrow = ingest == "arena-narrow"
    ingest = "arena" if narrow else ingest
    L = PackedLayout(cfg.num_fields, cfg.vocab_size if narrow else 0)
    B = 1024
    ex = ShardExecutor(m, L, [B], cuda, slots=3)
    eng = FanoutEngine(ex, DistContext(device=cuda), mode=mode, ingest=ingest,
                       arena=ArenaLayout(cfg.num_fields, max_rows=B), force_fanout=True)
    eng.prepare(B)
    assert eng.native_fanout_active
    for seed in range(4):  # cycles through every slot
        assert eng.self_check(B, seed=seed, slot=seed % 3)
    assert eng.native_fanout_active
    assert eng.comm_error() is None

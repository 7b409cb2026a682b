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
def test_native_serving_loop(cuda, mode, raw):
    """The C++ ServingLoop (parse -> H2D + step graph / fan-out -> encode) over a
    ring of request arenas; the last step's scores match a local forward.
    raw=False: packed varint requests, decoded on the GPU (the local replay
    skips the varint kernel for steps without any)."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.ops import hip, native

    cfg = ModelConfig(family="deepfm", vocab_size=50_000)
    m = build_model(cfg, cuda)
    F = cfg.num_fields
    L = PackedLayout(F)
    B, S, R = 1024, 4, 4
    ex = ShardExecutor(m, L, [B], cuda, slots=S)
    AL = ArenaLayout(F, max_rows=B)
    eng = FanoutEngine(ex, DistContext(device=cuda), mode="alltoall" if mode == "local" else mode, ingest="arena",
                       arena=AL, force_fanout=mode != "local")
    loop = hip().ServingLoop(eng.runner(), dict(depth=S - 1, fields=F, max_rows=B, version=1,
                                                        varint_chunks=AL.varint_chunks), eng.loop_slots(B))
    synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=5)
    inputs = []
    for p in range(5):
        ids, wts = synth.arrays(B)
        ids, wts = torch.from_numpy(ids), torch.from_numpy(wts)
        reqs = [native().encode_predict_request("DCN", "serving_default", None,
                                                [("feat_ids", ids[i:i + B // R]), ("feat_wts", wts[i:i + B // R])],
                                                raw or p == 1)
                for i in range(0, B, B // R)]
        ar = AL.alloc(pin=True)
        loop.add_input(ar, AL.place(ar, reqs))
        inputs.append((ids, wts))
    n = 11
    st = loop.run(n, True)
    assert st["errors"] == 0 and st["requests"] == n * R and st["rows"] == n * B
    assert st["response_bytes"] > n * B * 4 and len(st["latency_us"]) == n
    # every step's scores as the encoder read them: replays of one input agree
    sums = st["score_sum"]
    assert len(sums) == n
    for k in range(len(inputs), n):
        assert abs(sums[k] - sums[k - len(inputs)]) <= 1e-6 * max(1.0, abs(sums[k])), (k, sums)
    last = n - 1
    ids, wts = inputs[last % len(inputs)]
    got = eng.host_out(B, last % S)[:B].clone()
    want = m(ids.to(cuda), wts.to(cuda)).float().cpu()
    assert (got - want).abs().max().item() < 1e-5


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

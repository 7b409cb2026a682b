"""Embedding-parallel DLRM as a native two-lane step program on one GPU
(parallel/step_program.py, StepRunner.launch_program): a 1-rank sharded DLRM
(table-wise, row-wise and mixed placements; the exchanges are 1-rank RCCL
collectives on the aux lane) against the unsharded model, the route and mapped
interaction kernels against their fp32 CPU references, and the live server
serving requests through the captured program."""
import pytest
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import ModelConfig, ServingConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.parallel.dist import DistContext
from distributed_tf_serving_amd.parallel.embedding_sharding import (Placement, ShardedDLRM, ShardingPlan,
                                                                    dlrm_tables, plan_sharding)
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine
from distributed_tf_serving_amd.serving.arena import ArenaLayout
from distributed_tf_serving_amd.serving.executor import ShardExecutor
from distributed_tf_serving_amd.serving.packing import PackedLayout

pytestmark = pytest.mark.gpu


def _cfg():
    return ModelConfig(family="dlrm", num_fields=43, num_dense=13, table_rows=200_003, embed_dim=64,
                       bottom_mlp=(512, 256, 64), mlp_dims=(1024, 512, 256))


def _plan(cfg, policy):
    """1-rank plan; plan_sharding never picks row-wise at world 1, so the
    row-wise placements are written out (the rank owns every row range)."""
    base = plan_sharding(dlrm_tables(cfg), 1, policy="table")
    row = {"table": lambda t: False, "row": lambda t: True, "mixed": lambda t: t % 3 == 0}[policy]
    pl = [Placement(p.table, "row", ranges=[(0, cfg.table_rows)]) if row(p.table) else p for p in base.placements]
    return ShardingPlan(base.tables, 1, pl, base.budget_bytes)


def test_shard_route_matches_cpu(cuda):
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 1 << 40, (300, 43), generator=g)
    W, tm = 3, 4
    col = torch.randint(0, 43, (W * tm,), generator=g, dtype=torch.int64).to(torch.int32)
    mod = torch.randint(1, 10_000, (W * tm,), generator=g)
    off = torch.randint(0, 1 << 20, (W * tm,), generator=g)
    want = ops.shard_route(ids, W, tm, col, mod, off)
    got = ops.shard_route(ids.to(cuda), W, tm, col.to(cuda), mod.to(cuda), off.to(cuda))
    torch.cuda.synchronize()
    assert got.shape == (W, 300, tm) and torch.equal(got.cpu(), want)


def test_dot_interaction_table_map_matches_cpu(cuda):
    g = torch.Generator().manual_seed(4)
    B, T, D = 257, 30, 64
    dense = (torch.rand(B, D, generator=g) - 0.5).to(torch.bfloat16)
    flat = (torch.rand(3 * B * 11 + 7, D, generator=g) - 0.5).to(torch.bfloat16)
    off = torch.randint(0, 3 * B, (T,), generator=g)
    stride = torch.randint(1, 11, (T,), generator=g)
    want = ops.dot_interaction(dense, flat, 0, off, stride).float()
    got = ops.dot_interaction(dense.to(cuda), flat.to(cuda), 0, off.to(cuda), stride.to(cuda))
    torch.cuda.synchronize()
    assert (got.float().cpu() - want).abs().max().item() < 2e-2


@pytest.mark.parametrize("policy", ["table", "row", "mixed"])
def test_sharded_dlrm_one_rank_matches_unsharded(cuda, policy):
    cfg = _cfg()
    ctx = DistContext(device=cuda)
    m = ShardedDLRM(cfg, ctx, device=cuda, plan=_plan(cfg, policy)).eval()
    ref = build_model(cfg, cuda)
    g = torch.Generator().manual_seed(11)
    ids = torch.randint(0, 1 << 40, (700, cfg.num_fields), generator=g).to(cuda)
    wts = torch.rand(700, cfg.num_fields, generator=g).to(cuda)
    got, want = m(ids, wts), ref(ids, wts)
    torch.cuda.synchronize()
    assert (got - want).abs().max().item() < 1e-5


@pytest.mark.parametrize("policy", ["table", "mixed"])
def test_step_program_engine_and_live_server(cuda, policy):
    """FanoutEngine captures the program per slot; StepRunner.launch_program
    runs it (self_check vs the eager forward), then the native live server
    serves requests through it."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.live import LiveScheduler
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    cfg = _cfg()
    ctx = DistContext(device=cuda)
    m = ShardedDLRM(cfg, ctx, device=cuda, plan=_plan(cfg, policy)).eval()
    F, B, S = cfg.num_fields, 1024, 3
    ex = ShardExecutor(m, PackedLayout(F), [B], cuda, slots=S)
    eng = FanoutEngine(ex, ctx, mode="local", ingest="arena", arena=ArenaLayout(F, max_rows=B))
    eng.prepare(B)
    assert eng.program_active and eng.lockstep is False
    assert eng.self_check(B, seed=2)
    sc = ServingConfig(max_batch_rows=B, allowed_batch_sizes=(B,), batch_timeout_us=100)
    live = LiveScheduler(eng, sc, buckets=[B], depth=S)
    try:
        synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=9)
        for rows in (1, 300, 1024):
            req = synth.serialized(rows, raw=True)
            r = pb.PredictRequest.FromString(req)
            ids = torch.from_numpy(T.to_ndarray(r.inputs["feat_ids"])).to(cuda)
            wts = torch.from_numpy(T.to_ndarray(r.inputs["feat_wts"])).to(cuda)
            want = m(ids, wts).float().cpu()
            resp = pb.PredictResponse.FromString(live.predict_bytes(req, 30.0))
            got = torch.from_numpy(T.to_ndarray(resp.outputs["prediction_node"]))
            assert got.shape == (rows,)
            assert (got - want).abs().max().item() < 1e-5
    finally:
        live.close()


def test_dlrm_multi_hot_gpu_matches_cpu(cuda):
    """K1b bag kernel inside the multi-hot DLRM forward: GPU vs the fp32 CPU
    model with the same weights."""
    cfg = ModelConfig(family="dlrm", num_fields=13 + 15 * 2, num_dense=13, table_rows=50_021, embed_dim=64,
                      multi_hot=2, bottom_mlp=(512, 256, 64), mlp_dims=(1024, 512, 256))
    gm, cm = build_model(cfg, cuda), build_model(cfg, "cpu")
    cm.load_state_dict({k: v.detach().cpu() for k, v in gm.state_dict().items()})  # device RNG streams differ
    g = torch.Generator().manual_seed(6)
    ids = torch.randint(0, 1 << 40, (513, cfg.num_fields), generator=g)
    wts = torch.rand(513, cfg.num_fields, generator=g)
    got = gm(ids.to(cuda), wts.to(cuda)).float().cpu()
    want = cm(ids, wts).float()
    assert (got - want).abs().max().item() < 2e-2


def test_gather_gemm_resolved_on_another_stream_is_identical(cuda):
    """embed_gemm_resolve + embed_gemm(resolved=...) (the resolve pass moved to
    the step program's aux lane) gives bit-identical results to the one-call
    gather-GEMM."""
    g = torch.Generator().manual_seed(5)
    B, F, V, N = 16384, 43, 100_003, 1024
    table = ((torch.rand(V, 64, generator=g) - 0.5) * 0.2).to(torch.bfloat16).to(cuda)
    lin = ((torch.rand(V, generator=g) - 0.5) * 0.02).to(cuda)
    W = ((torch.rand(N, F * 64, generator=g) - 0.5) * 0.05).to(torch.bfloat16).to(cuda)
    b = ((torch.rand(N, generator=g) - 0.5) * 0.1).to(cuda)
    ids = torch.randint(0, 1 << 40, (B, F), generator=g).to(cuda)
    wts = torch.rand(B, F, generator=g).to(cuda)
    h0, p0 = ops.embed_gemm(table, ids, wts, lin, V, 0.25, W, b, "relu", fm2=True)
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):
        r = ops.embed_gemm_resolve(table, ids, wts, lin, V, 0.25, True)
    torch.cuda.current_stream(cuda).wait_stream(side)
    h1, p1 = ops.embed_gemm(table, ids, wts, lin, V, 0.25, W, b, "relu", fm2=True, resolved=r)
    torch.cuda.synchronize()
    assert torch.equal(h0, h1) and torch.equal(p0[:, :B], p1[:, :B])


def test_resolve_lane_program_engine_and_live_server(cuda, monkeypatch):
    """A local step at the gather-GEMM bucket runs as a two-lane program with
    DTFS_RESOLVE_LANE=1 (resolve on the aux lane after the H2D, the compute
    lane waits only for it), the small bucket as the one-stream step;
    self-check and served requests match the model. DCN v1: DeepFM and
    Wide&Deep resolve their rows inside the one-launch tower (no pass to move)."""
    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.serving.live import LiveScheduler
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    monkeypatch.setenv("DTFS_RESOLVE_LANE", "1")
    cfg = ModelConfig(family="dcn", vocab_size=100_003, embed_dim=64, mlp_dims=(1024, 512, 256))
    m = build_model(cfg, cuda)
    F, S = cfg.num_fields, 3
    buckets = [2048, 16384]
    ex = ShardExecutor(m, PackedLayout(F), buckets, cuda, slots=S)
    eng = FanoutEngine(ex, DistContext(device=cuda), mode="local", ingest="arena", arena=ArenaLayout(F, max_rows=16384))
    for B in buckets:
        eng.prepare(B)
    assert eng.program_active and eng._cprog is None and eng._program_buckets == {16384}
    kinds = [o["kind"] for o in eng._programs[(16384, 0)].spec["ops"]]
    assert kinds == ["kernels", "kernels", "record", "wait", "kernels"], kinds  # varints, resolve | forward
    for B in buckets:
        assert eng.self_check(B, seed=3)
    sc = ServingConfig(max_batch_rows=16384, allowed_batch_sizes=tuple(buckets), batch_timeout_us=100)
    live = LiveScheduler(eng, sc, buckets=buckets, depth=S)
    try:
        synth = SyntheticRequests(fields=F, id_space=1 << 40, dist="zipf", seed=19)
        reqs = [synth.serialized(512, raw=True) for _ in range(40)]  # > 16384 rows: full gather-GEMM steps
        import concurrent.futures as cf

        with cf.ThreadPoolExecutor(8) as pool:
            outs = list(pool.map(lambda q: live.predict_bytes(q, 30.0), reqs))
        for req, out in zip(reqs, outs):
            r = pb.PredictRequest.FromString(req)
            ids = torch.from_numpy(T.to_ndarray(r.inputs["feat_ids"])).to(cuda)
            wts = torch.from_numpy(T.to_ndarray(r.inputs["feat_wts"])).to(cuda)
            want = m(ids, wts).float().cpu()
            got = torch.from_numpy(T.to_ndarray(pb.PredictResponse.FromString(out).outputs["prediction_node"]))
            assert (got - want).abs().max().item() < 5e-3  # 512-row forward vs rows inside a 16384-row step
    finally:
        live.close()

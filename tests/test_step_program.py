"""Step programs on CPU (parallel/step_program.py): lane/event validation (the
Python mirror of StepProgram::validate), the routing and table-map references
the GPU kernels are checked against, and a 1-rank sharded DLRM (every
placement kind) against the unsharded model."""
import pytest
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.parallel import step_program as sp
from distributed_tf_serving_amd.parallel.dist import DistContext
from distributed_tf_serving_amd.parallel.embedding_sharding import (Placement, ShardedDLRM, ShardingPlan,
                                                                    dlrm_tables, plan_sharding)


def _k(lane):
    return sp.Kernels(lane, lambda: None)


def test_validate_requires_join():
    sp.validate([_k(sp.COMPUTE)])
    sp.validate([_k(sp.AUX), sp.Sync("record", sp.AUX, 0), sp.Sync("wait", sp.COMPUTE, 0), _k(sp.COMPUTE)])
    with pytest.raises(ValueError, match="not joined"):
        sp.validate([_k(sp.AUX)])
    with pytest.raises(ValueError, match="not joined"):  # aux work after the last join
        sp.validate([_k(sp.AUX), sp.Sync("record", sp.AUX, 0), sp.Sync("wait", sp.COMPUTE, 0), _k(sp.AUX)])
    with pytest.raises(ValueError, match="before it is recorded"):
        sp.validate([sp.Sync("wait", sp.COMPUTE, 1)])
    with pytest.raises(ValueError, match="out of range"):
        sp.validate([sp.Sync("record", sp.AUX, 9)])


def test_shard_route_reference():
    ids = torch.tensor([[5, 17, 40], [-3, 8, 100]])
    col = torch.tensor([2, 0, 1, 1], dtype=torch.int32)
    mod = torch.tensor([7, 10, 3, 1])
    off = torch.tensor([100, 0, 50, 9])
    out = ops.shard_route(ids, 2, 2, col, mod, off)
    assert out.dtype == torch.int32 and out.shape == (2, 2, 2)
    # owner 0 slots (col 2 mod 7 +100, col 0 mod 10), owner 1 slots (col 1 mod 3 +50, pad)
    assert out[0].tolist() == [[100 + 40 % 7, 5], [100 + 100 % 7, (-3) % 10]]
    assert out[1].tolist() == [[50 + 17 % 3, 9], [50 + 8 % 3, 9]]


def test_dot_interaction_map_equals_dense_layout():
    g = torch.Generator().manual_seed(1)
    B, T = 9, 5
    emb = torch.rand(B, T, 64, generator=g).to(torch.bfloat16)
    dense = torch.rand(B, 64, generator=g).to(torch.bfloat16)
    want = ops.dot_interaction(dense, emb)
    # the same vectors in an all-to-all style layout [owner][b][slot] with 2 slots
    flat = torch.zeros(3 * B * 2, 64, dtype=torch.bfloat16)
    off, stride = [], []
    for t in range(T):
        s, j = t // 2, t % 2
        for b in range(B):
            flat[s * B * 2 + b * 2 + j] = emb[b, t]
        off.append(s * B * 2 + j)
        stride.append(2)
    got = ops.dot_interaction(dense, flat, 0, torch.tensor(off), torch.tensor(stride))
    assert torch.equal(got, want)


@pytest.mark.parametrize("policy", ["table", "row", "mixed"])
def test_sharded_dlrm_one_rank_cpu(policy):
    cfg = ModelConfig(family="dlrm", num_fields=20, num_dense=5, table_rows=997, embed_dim=64,
                      bottom_mlp=(32, 64), mlp_dims=(64, 32))
    base = plan_sharding(dlrm_tables(cfg), 1, policy="table")
    row = {"table": lambda t: False, "row": lambda t: True, "mixed": lambda t: t % 2 == 1}[policy]
    plan = ShardingPlan(base.tables, 1, [Placement(p.table, "row", ranges=[(0, cfg.table_rows)])
                                        if row(p.table) else p for p in base.placements], base.budget_bytes)
    m = ShardedDLRM(cfg, DistContext(), plan=plan)
    ref = build_model(cfg)
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, 10 ** 12, (13, cfg.num_fields), generator=g)
    wts = torch.rand(13, cfg.num_fields, generator=g)
    assert (m(ids, wts) - ref(ids, wts)).abs().max().item() < 1e-5
    ops_ = m.build_program(ids, wts, 13, m.alloc(13))
    sp.validate(ops_)
    # one rank: the table-wise all-to-alls are the identity (the buffers
    # alias) and leave the program; row-wise tables keep their all-gather /
    # reduce-scatter pair (multi-rank programs: test_embedding_sharding)
    kinds = [o.kind for o in ops_ if isinstance(o, sp.Coll)]
    assert kinds == ([] if policy == "table" else ["allgather", "reduce_scatter"])
    assert m.exchange_bytes(13) == 0


def test_dlrm_multi_hot_bag_matches_manual_pooling():
    """Multi-hot DLRM (K1b): table t's `hot` ids are hashed onto its rows and
    sum-pooled with their feat_wts; checked against explicit row gathers."""
    cfg = ModelConfig(family="dlrm", num_fields=13 + 15 * 2, num_dense=13, table_rows=1009, embed_dim=64,
                      multi_hot=2, bottom_mlp=(32, 64), mlp_dims=(64, 32))
    m = build_model(cfg)
    assert m.T == 15 and m.hot == 2
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 10 ** 12, (6, cfg.num_fields), generator=g)
    wts = torch.rand(6, cfg.num_fields, generator=g)
    got = m.lookup(ids, wts).float()
    want = torch.zeros(6, 15, 64)
    for b in range(6):
        for t in range(15):
            for h in range(2):
                c = 13 + 2 * t + h
                row = t * 1009 + int(ids[b, c]) % 1009
                want[b, t] += m.emb[row].float() * wts[b, c]
    assert (got - want).abs().max().item() < 2e-2  # bf16 pooled output
    y = m(ids, wts)
    assert y.shape == (6,) and torch.isfinite(y).all()
    with pytest.raises(ValueError):
        build_model(ModelConfig(family="dlrm", num_fields=42, num_dense=13, multi_hot=2))

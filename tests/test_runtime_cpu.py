"""Host runtime: dynamic batcher, candidate splitter, models on CPU, step pipeline."""
import threading
import time

import numpy as np
import pytest
import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.config import ModelConfig, list_presets, load_preset
from distributed_tf_serving_amd.models import FAMILIES, build_model
from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.parallel.dist import DistContext, reference_partition, split_rows
from distributed_tf_serving_amd.parallel.fanout import FanoutEngine
from distributed_tf_serving_amd.serving.executor import ShardExecutor
from distributed_tf_serving_amd.serving.packing import PackedLayout


# ------------------------------------------------------------------ batcher
def test_batcher_full_batch_and_order():
    b = native().DynamicBatcher(100, 1_000_000, 0)
    for t in range(5):
        assert b.submit(t, 30)
    batch = b.next_batch(0)
    assert [i.ticket for i in batch.items] == [0, 1, 2] and batch.rows == 90  # never split, never overflow
    batch = b.next_batch(0)  # 60 rows left < 100 and the timeout is 1 s: nothing ready
    assert batch.items == [] and not batch.closed
    b.close()
    batch = b.next_batch(0)
    assert [i.ticket for i in batch.items] == [3, 4]
    assert b.next_batch(0).closed


def test_batcher_eager_when_idle():
    b = native().DynamicBatcher(100, 10_000_000, 0)  # 10 s batch timeout
    b.submit(1, 10)
    b.submit(2, 20)
    assert b.next_batch(0).items == []  # not full, timeout far away
    t = time.perf_counter()
    batch = b.next_batch(0, True)  # idle device: take what is queued now
    assert [i.ticket for i in batch.items] == [1, 2] and batch.rows == 30
    assert time.perf_counter() - t < 0.5
    b.close()


def test_batcher_timeout_and_oversize():
    b = native().DynamicBatcher(64, 2000, 0)
    b.submit(1, 10)
    t = time.perf_counter()
    batch = b.next_batch(1_000_000)
    assert [i.ticket for i in batch.items] == [1]
    assert time.perf_counter() - t < 0.5
    b.submit(2, 500)  # larger than max batch: served alone
    b.submit(3, 5)
    assert [i.ticket for i in b.next_batch(1_000_000).items] == [2]
    st = b.stats()
    assert st.submitted == 3 and st.batches == 2


def test_batcher_deadline_and_backpressure():
    nat = native()
    b = nat.DynamicBatcher(1000, 50_000, 100)
    assert b.submit(1, 60, nat.now_us() + 1)  # expires almost immediately
    assert not b.submit(2, 60)  # would exceed max_queued_rows=100
    time.sleep(0.01)
    batch = b.next_batch(1000)
    assert [i.ticket for i in batch.expired] == [1] and batch.items == []
    assert b.submit(3, 60)


def test_batcher_concurrent_producers():
    b = native().DynamicBatcher(256, 500, 0)
    n = 200

    def prod(base):
        for i in range(n):
            b.submit(base + i, 4)

    ths = [threading.Thread(target=prod, args=(k * 1000,)) for k in range(4)]
    [t.start() for t in ths]
    got = []
    while len(got) < 4 * n:
        batch = b.next_batch(100_000)
        assert batch.rows <= 256
        got += [i.ticket for i in batch.items]
    [t.join() for t in ths]
    assert sorted(got) == sorted(k * 1000 + i for k in range(4) for i in range(n))


# ------------------------------------------------------------------ splitter
@pytest.mark.parametrize("n", [0, 1, 187, 1500])
@pytest.mark.parametrize("parts", range(1, 9))
def test_split_rows(n, parts):
    s = split_rows(n, parts)
    assert len(s) == parts and sum(k for _, k in s) == n
    assert all(s[i][0] + s[i][1] == s[i + 1][0] for i in range(parts - 1))
    sizes = [k for _, k in s]
    assert max(sizes) - min(sizes) <= 1


def test_reference_partition_bug_documented():
    # reference DCNClient.java:46-55 splits the flat 43-per-row list: at N=8 the
    # shard element counts are not multiples of 43
    flat = list(range(1500 * 43))
    parts = reference_partition(flat, 8)
    assert [len(p) for p in parts][:2] == [8062, 8062] and len(parts[-1]) == 8066
    assert any(len(p) % 43 for p in parts)


# ------------------------------------------------------------------ config
def test_presets_load():
    names = list_presets()
    assert {"wdl_tiny_cpu", "deepfm_1gpu", "deepfm_fanout4", "dlrm_sharded8", "dcn_v2_fp8", "reference_dcn"} <= set(names)
    for n in names:
        cfg = load_preset(n)
        assert cfg.model.family in FAMILIES
    assert load_preset("dcn_v2_fp8").model.gemm_dtype == "fp8"
    assert load_preset("dlrm_sharded8").model.table_rows == 100_000_000


# ------------------------------------------------------------------ models
def small_cfg(family, **kw):
    base = dict(family=family, vocab_size=5000, table_rows=500, embed_dim=64 if family == "dlrm" else 16,
                mlp_dims=(64, 32), bottom_mlp=(32, 64), num_cross_layers=2)
    base.update(kw)
    return ModelConfig(**base)


@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_model_forward_cpu(family):
    m = build_model(small_cfg(family))
    ids = torch.randint(-10**12, 10**12, (7, 43))
    wts = torch.rand(7, 43)
    y = m(ids, wts)
    assert y.shape == (7,) and y.dtype == torch.float32
    assert ((y > 0) & (y < 1)).all()
    # deterministic given the seed
    y2 = build_model(small_cfg(family))(ids, wts)
    assert torch.equal(y, y2)
    # row independence: scoring a row alone gives the same CTR
    assert torch.allclose(m(ids[3:4], wts[3:4]), y[3:4], atol=1e-6)


def test_model_signature():
    m = build_model(small_cfg("dcn"))
    sig = m.signature()
    assert sig["inputs"]["feat_ids"] == ("DT_INT64", [-1, 43])
    assert "prediction_node" in sig["outputs"]


def test_fm_identity_against_bruteforce():
    table = torch.randn(50, 8)
    ids = torch.randint(0, 50, (4, 6))
    wts = torch.rand(4, 6)
    _, fm = ops.embed(table, ids, wts, want_x=False, want_fm=True, fm2=True, modulo=50)
    e = table[ids] * wts[..., None]
    brute = torch.zeros(4)
    for i in range(6):
        for j in range(i + 1, 6):
            brute += (e[:, i] * e[:, j]).sum(-1)
    assert torch.allclose(fm, brute, atol=1e-4)


def test_dlrm_interaction_layout():
    dense = torch.randn(3, 64)
    emb = torch.randn(3, 4, 64)
    z = ops.dot_interaction(dense, emb)
    assert z.shape[1] == ops.interaction_cols(4) and z.shape[1] % 8 == 0
    X = torch.cat([dense[:, None], emb], 1)
    assert torch.allclose(z[:, 64], (X[:, 1] * X[:, 0]).sum(-1), atol=1e-4)
    assert torch.allclose(z[:, 64 + 1], (X[:, 2] * X[:, 0]).sum(-1), atol=1e-4)
    assert torch.allclose(z[:, 64 + 2], (X[:, 2] * X[:, 1]).sum(-1), atol=1e-4)
    assert (z[:, 64 + 10:] == 0).all()


def test_sort_scores_cpu():
    s = torch.tensor([0.3, 0.1, 0.3, 0.9])
    v, p = ops.sort_scores(s)
    assert v.tolist() == sorted(s.tolist()) and p.tolist() == [1, 0, 2, 3]
    v, p = ops.sort_scores(s, descending=True, k=2)
    assert p.tolist() == [3, 0]


# ------------------------------------------------------------------ executor / engine / pipeline (CPU)
def test_executor_and_local_engine_cpu():
    m = build_model(small_cfg("deepfm"))
    L = PackedLayout(43)
    ex = ShardExecutor(m, L, [8, 16], "cpu", slots=2)
    eng = FanoutEngine(ex, DistContext(), mode="alltoall")
    assert eng.mode == "local"  # world 1
    ids = torch.randint(0, 10**9, (16, 43))
    wts = torch.rand(16, 43)
    buf = eng.host_in(16, 1)
    L.ids(buf).copy_(ids)
    L.wts(buf).copy_(wts)
    h = eng.launch(16, 1)
    out = h.wait()
    assert torch.allclose(out, m(ids, wts), atol=1e-6)
    assert torch.allclose(ex.run_rows(ids[:5], wts[:5]), m(ids[:5], wts[:5]), atol=1e-6)

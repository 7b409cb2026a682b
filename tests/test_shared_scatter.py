"""Shared-arena scatter (csrc/runtime/shared_scatter.h): the plan rank 0
publishes and the share copies every rank makes, checked on the host against
a full unpack of the same arena (the GPU kernels read rows through the same
row table). Multi-process serving over it: tests/test_cluster_server.py."""
import os
import secrets

import numpy as np
import pytest
import torch

from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.arena import ArenaLayout
from distributed_tf_serving_amd.serving.packing import PackedLayout
from distributed_tf_serving_amd.wire import schema as pb
from distributed_tf_serving_amd.wire.tensor import make_tensor_proto


def _requests(rng, sizes, F):
    """Requests of the given row counts in three encodings: raw
    tensor_content, packed int64_val varints + float_val (the reference
    client's), int32 ids."""
    out = []
    for i, n in enumerate(sizes):
        ids = rng.integers(0, 1 << 40, size=(n, F), dtype=np.int64)
        wts = rng.random((n, F), dtype=np.float32)
        kind = i % 3
        if kind == 0:
            out.append(native().encode_predict_request("DCN", "serving_default", None,
                                                       [("feat_ids", torch.from_numpy(ids)),
                                                        ("feat_wts", torch.from_numpy(wts))], True))
            continue
        req = pb.PredictRequest()
        req.model_spec.name = "DCN"
        if kind == 1:
            t = req.inputs["feat_ids"]
            t.dtype = 9  # DT_INT64
            t.tensor_shape.dim.add().size = n
            t.tensor_shape.dim.add().size = F
            t.int64_val.extend(ids.reshape(-1).tolist())
            w = req.inputs["feat_wts"]
            w.dtype = 1
            w.tensor_shape.dim.add().size = n
            w.tensor_shape.dim.add().size = F
            w.float_val.extend(wts.reshape(-1).tolist())
        else:
            req.inputs["feat_ids"].CopyFrom(make_tensor_proto((ids % (1 << 31)).astype(np.int32)))
            req.inputs["feat_wts"].CopyFrom(make_tensor_proto(wts))
        out.append(req.SerializeToString())
    return out


@pytest.mark.parametrize("world,sizes", [(1, [5, 9]), (2, [32, 32, 32, 32]), (2, [7, 50, 1, 3, 60]),
                                         (3, [40, 1, 1, 33, 17, 30]), (4, [100, 3, 4, 5, 6, 7, 8, 9])])
def test_shares_reproduce_every_rank_slice(world, sizes):
    F, B = 6, 64
    rows = sum(sizes)
    assert rows <= world * B
    lay = ArenaLayout(F, max_rows=world * B, gpu_varint=False)
    name = f"/dtfs-test-sct-{os.getpid()}-{secrets.token_hex(4)}"
    segs = [native().SharedScatter(name, world, 0, True, F, 2, lay.capacity, 2, world * B)]
    segs += [native().SharedScatter(name, world, r, False) for r in range(1, world)]
    segs[0].unlink()
    assert segs[0].all_attached
    rng = np.random.default_rng(world * 100 + len(sizes))
    ar = segs[0].arena(1)
    ab = lay.build(ar, lay.place(ar, _requests(rng, sizes, F)))
    assert ab.total_rows == rows and all(e == "" for e in ab.errors), ab.errors
    pl = PackedLayout(F)
    full = lay.unpack_cpu(ar, pl.alloc(world * B))
    shares = native().SharedScatter.shares(ar, F, world, B)
    k = segs[0].begin_step()
    segs[0].publish_plan(k, 1, B)
    copied = 0
    for r, s in enumerate(segs):
        if r:
            assert s.begin_step() == k
        loc = lay.alloc()
        row0, n, nbytes = s.take_share(k, loc, 5.0)
        assert (row0, n) == (shares[r][0], shares[r][1])
        per = -(-rows // world)  # even split over the ranks
        assert row0 == min(rows, r * per) and n == max(0, min(per, rows - r * per)) and n <= B
        got = lay.unpack_cpu(loc, pl.alloc(B))
        assert torch.equal(got[:n], full[row0: row0 + n]), f"rank {r}"
        assert not got[n:].any()  # padding rows read nothing
        copied += nbytes
        s.out(0)[r * B: r * B + n] = got[:n, 0].float()  # "scores": the rank's fixed output slice
        s.mark_done(k)
    ok, err = segs[0].wait_done(k, 1.0)
    assert ok, err
    segs[0].compact_scores(k, 0)  # rank r's rows move from r * B to their batch rows
    assert torch.equal(segs[0].out(0)[:rows], full[:rows, 0].float())
    # every rank copied only its share: together about one batch, not world x
    assert copied <= ab.used_bytes + world * (64 + 8 * 4096), (copied, ab.used_bytes)
    assert all(len(sh[2]) <= 8 for sh in shares)


def test_wait_done_names_the_late_rank():
    F = 4
    lay = ArenaLayout(F, max_rows=32, gpu_varint=False)
    name = f"/dtfs-test-sct-{os.getpid()}-{secrets.token_hex(4)}"
    s0 = native().SharedScatter(name, 2, 0, True, F, 2, lay.capacity, 2, 32)
    s1 = native().SharedScatter(name, 2, 1, False)
    s0.unlink()
    s0.mark_done(0)
    ok, err = s0.wait_done(0, 0.05)
    assert not ok and "rank 1" in err
    s1.mark_done(0)
    assert s0.wait_done(0, 0.05)[0]


def test_gpu_varint_arena_is_refused():
    F = 4
    lay = ArenaLayout(F, max_rows=16, gpu_varint=True)
    ar = lay.alloc()
    rng = np.random.default_rng(0)
    reqs = _requests(rng, [4, 4], F)  # the second one: packed varints, left to the GPU decode
    lay.build(ar, lay.place(ar, reqs))
    with pytest.raises(Exception, match="varint"):
        native().SharedScatter.shares(ar, F, 2, 8)


def test_numa_placement_puts_each_share_on_its_reader_node():
    """Per-rank NUMA slices of the shared arenas (a 2-socket node: ranks 0-1
    on node 0, ranks 2-3 on node 1): rank r's share of every arena, about
    payload [r S, (r + 1) S) of a full batch, is bound to r's node - the last
    rank's slice runs to the arena's end; nothing is bound for ranks on rank
    0's node. On a one-node machine the binding reports failure (best effort)
    and the segment serves as before."""
    F, world, B = 6, 4, 64
    lay = ArenaLayout(F, max_rows=world * B, gpu_varint=False)
    name = f"/dtfs-test-sct-{os.getpid()}-{secrets.token_hex(4)}"
    expected = world * B * (12 * F + 16)
    seg = native().SharedScatter(name, world, 0, True, F, 3, lay.capacity, 2, world * B, -1, [0, 0, 1, 1], expected)
    try:
        pl = seg.placement()
        page = 4096
        stride = -(-lay.capacity // page) * page
        payload_off = 64 + 32 * 1024  # kArenaPayloadOff: header + request descriptors
        up = lambda x: -(-x // page) * page  # noqa: E731
        # per arena: ranks 2 and 3 (both node 1) merge into one slice from rank 2's
        # first page to the arena's end
        assert len(pl) == 3 and all(s["node"] == 1 and s["rank"] == 2 for s in pl), pl
        for s in pl:
            a0 = s["hi"] - stride  # the arena's start (its slice ends at the arena's end)
            assert a0 % page == 0 and s["lo"] - a0 == up(payload_off + expected * 2 // world)
        n_nodes = native().numa_node_count()
        if n_nodes < 2:
            assert not any(s["bound"] for s in pl)  # no node 1 here
        else:
            assert all(s["bound"] for s in pl)
            seg.arena(0)[pl[0]["lo"] - (pl[0]["hi"] - stride):].fill_(1)  # first touch places the pages
            assert seg.page_node(pl[0]["lo"]) == 1
        # every rank on node 0, or no expected payload: nothing placed
        name2 = name + "b"
        seg2 = native().SharedScatter(name2, world, 0, True, F, 3, lay.capacity, 2, world * B, -1, [0, 0, 0, 0],
                                      expected)
        assert seg2.placement() == []
        seg2.unlink()
        with pytest.raises(Exception):  # one node per rank
            native().SharedScatter(name + "c", world, 0, True, F, 3, lay.capacity, 2, world * B, -1, [0, 1], expected)
    finally:
        seg.unlink()


def test_placement_sizes_shares_from_the_narrowed_rows():
    """The per-rank NUMA ranges follow the bytes a share actually takes: GPU
    live servers narrow requests on the host (3-byte rows for tables of <= 2^24
    rows, weights, an 8-byte row-table entry), far below raw tensor_content."""
    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.parallel.shared_scatter import expected_row_bytes, live_narrowing

    assert expected_row_bytes(43) == 12 * 43 + 16
    assert expected_row_bytes(43, 1_000_000) == 3 * 43 + 4 * 43 + 8
    assert expected_row_bytes(43, 1 << 30) == 4 * 43 + 4 * 43 + 8
    assert expected_row_bytes(39, 1 << 20, narrow_wts_cols=13) == 3 * 39 + 4 * 13 + 8
    m = build_model(ModelConfig(family="deepfm", vocab_size=1000, embed_dim=16, num_fields=8, mlp_dims=[16]), "cpu")
    assert live_narrowing(m, cuda=False) == (0, 0)  # CPU servables do not narrow
    assert live_narrowing(m, cuda=True) == (1000, 0)
    assert live_narrowing(m, cuda=True, narrow=False) == (0, 0)

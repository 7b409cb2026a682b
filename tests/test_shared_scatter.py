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

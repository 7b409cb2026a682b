"""Request arena host build (csrc/runtime/arena.cpp) on the CPU: raw and packed
requests, GPU varint chunk tables checked through the host reference of the
varint kernel, and the host-decode fallback."""
import pytest
import torch

from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.serving.arena import ArenaLayout
from distributed_tf_serving_amd.serving.packing import PackedLayout

F = 43


def _req(ids, wts, raw):
    return native().encode_predict_request("DCN", "serving_default", None, [("feat_ids", ids), ("feat_wts", wts)],
                                           raw)


def _ids(kind, n, g):
    if kind == "small":
        return torch.randint(1, 100, (n, F), generator=g)
    if kind == "neg":
        return torch.randint(-(1 << 62), 1 << 62, (n, F), generator=g)
    return torch.randint(0, 1 << 40, (n, F), generator=g) >> torch.randint(0, 40, (n, F), generator=g)


@pytest.mark.parametrize("gpu_varint", [True, False])
def test_arena_mixed_requests_roundtrip(gpu_varint):
    g = torch.Generator().manual_seed(11)
    A, L = ArenaLayout(F, 4096, gpu_varint=gpu_varint), PackedLayout(F)
    ar = A.alloc()
    reqs, ids_l, wts_l = [], [], []
    for n, kind, raw in ((700, "mixed", False), (1, "small", False), (250, "mixed", True), (900, "neg", False),
                         (333, "small", False)):
        ids, wts = _ids(kind, n, g), torch.rand(n, F, generator=g)
        reqs.append(_req(ids, wts, raw))
        ids_l.append(ids)
        wts_l.append(wts)
    ab = A.build(ar, A.place(ar, reqs))
    assert not any(ab.errors) and ab.total_rows == 2184
    assert ab.n_gpu_varint == (4 if gpu_varint else 0)
    assert ab.n_decoded == (0 if gpu_varint else 4)
    got = A.unpack_cpu(ar, L.alloc(ab.total_rows))
    assert torch.equal(L.ids(got), torch.cat(ids_l))
    assert torch.equal(L.wts(got), torch.cat(wts_l))


def test_arena_gpu_varint_copies_fewer_bytes():
    # the point of the GPU decode: the H2D copy holds wire bytes, not int64 ids
    g = torch.Generator().manual_seed(5)
    ids, wts = _ids("small", 512, g), torch.rand(512, F, generator=g)
    sizes = {}
    for gv in (True, False):
        A = ArenaLayout(F, 1024, gpu_varint=gv)
        ar = A.alloc()
        sizes[gv] = A.build(ar, A.place(ar, [_req(ids, wts, False)])).used_bytes
    assert sizes[True] < sizes[False] - 512 * F * 7


def test_arena_varint_chunk_capacity_falls_back_to_host():
    # a request whose chunks do not fit the table is decoded on the host
    g = torch.Generator().manual_seed(2)
    ids, wts = _ids("neg", 200, g), torch.rand(200, F, generator=g)
    A, L = ArenaLayout(F, 1024), PackedLayout(F)
    ar = A.alloc()
    spans = A.place(ar, [_req(ids, wts, False)])
    ab = native().arena_build(ar, spans, "feat_ids", "feat_wts", F, 1024, 3)  # needs 21 chunks
    assert ab.n_gpu_varint == 0 and ab.n_decoded == 1
    got = A.unpack_cpu(ar, L.alloc(200))
    assert torch.equal(L.ids(got), ids)


def test_arena_bad_shape_is_a_request_error():
    g = torch.Generator().manual_seed(1)
    A = ArenaLayout(F, 1024)
    ar = A.alloc()
    bad = native().encode_predict_request("DCN", "serving_default", None,
                                          [("feat_ids", _ids("small", 4, g)[:, :40]),
                                           ("feat_wts", torch.rand(4, 40))], False)
    ok = _req(_ids("small", 3, g), torch.rand(3, F), False)
    ab = A.build(ar, A.place(ar, [bad, ok]))
    assert "shape" in ab.errors[0] and ab.errors[1] == "" and ab.total_rows == 3

"""Checkpoint / resume (safetensors): identical scores after a round trip;
sharded DLRM checkpoints written by 2 ranks load on 3 (re-sharding)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model
from distributed_tf_serving_amd.utils.checkpoint import load_model, read_config, save_model


@pytest.mark.parametrize("family", ["wdl", "deepfm", "dcn", "dcn_v2"])
def test_round_trip(tmp_path, family):
    cfg = ModelConfig(family=family, vocab_size=3000, embed_dim=16, mlp_dims=(32, 16), seed=5)
    m = build_model(cfg)
    p = str(tmp_path / "m.safetensors")
    save_model(m, p)
    assert read_config(p) == cfg
    other = build_model(ModelConfig(family=family, vocab_size=3000, embed_dim=16, mlp_dims=(32, 16), seed=99))
    ids = torch.randint(0, 1 << 40, (9, 43))
    wts = torch.rand(9, 43)
    assert not torch.allclose(other(ids, wts), m(ids, wts))
    load_model(other, p)
    assert torch.equal(other(ids, wts), m(ids, wts))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(seed):
    return ModelConfig(family="dlrm", num_fields=12, num_dense=3, table_rows=101, embed_dim=64, bottom_mlp=(32, 64),
                       mlp_dims=(64, 32), seed=seed)


def _worker(rank, world, port, phase, path, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from distributed_tf_serving_amd.parallel.dist import init_from_env, shutdown
    from distributed_tf_serving_amd.parallel.embedding_sharding import ShardedDLRM
    from distributed_tf_serving_amd.utils.checkpoint import load_sharded, save_sharded

    try:
        ctx = init_from_env(device="cpu")
        g = torch.Generator().manual_seed(17 + rank)
        ids = torch.randint(0, 1 << 40, (4, 12), generator=g)
        wts = torch.rand(4, 12, generator=g)
        if phase == "save":
            m = ShardedDLRM(_cfg(seed=1), ctx, policy="row" if world == 2 else "table")
            save_sharded(m, path)
            q.put((rank, "ok"))
        else:
            m = ShardedDLRM(_cfg(seed=2), ctx, policy="auto")  # different init, different plan
            load_sharded(m, path)
            ref = build_model(_cfg(seed=1))
            q.put((rank, float((m(ids, wts) - ref(ids, wts)).abs().max())))
        shutdown()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc()))


def _run(world, phase, path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, phase, path, q)) for r in range(world)]
    [p.start() for p in procs]
    out = dict(q.get(timeout=240) for _ in range(world))
    [p.join(timeout=60) for p in procs]
    return out


@pytest.mark.slow
def test_sharded_dlrm_checkpoint_reshards(tmp_path):
    path = str(tmp_path / "dlrm_ckpt")
    saved = _run(2, "save", path)
    assert all(v == "ok" for v in saved.values()), saved
    assert os.path.exists(os.path.join(path, "manifest.json"))
    loaded = _run(3, "load", path)
    for r, v in loaded.items():
        assert isinstance(v, float), f"rank {r}: {v}"
        assert v < 1e-5

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


@pytest.mark.parametrize("mode", ["alltoall", "scatter"])
@pytest.mark.parametrize("ingest", ["packed", "arena"])
def test_native_fanout_step_matches_local(cuda, mode, ingest):
    cfg = ModelConfig(family="deepfm", vocab_size=50_000)
    m = build_model(cfg, cuda)
    L = PackedLayout(cfg.num_fields)
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

"""One-shot peer exchange (csrc/kernels/peer.hip, RcclComm.peer_*): exact
alltoall / allgather / gather / scatter against the expected layout and against
RCCL, with 1 rank in-process and 2 / 3 ranks sharing the one GPU of the box
(IPC-mapped mailboxes between processes), plus the bounded-spin failure path
(a rank that never joins makes the others report a timeout, not hang)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_peer_exchange_single_rank(cuda):
    from distributed_tf_serving_amd.parallel.dist import DistContext
    from distributed_tf_serving_amd.parallel.native_comm import create_comm

    c = create_comm(DistContext(device=cuda), peer_cap=4096)
    assert c.peer_enabled and c.peer_cap >= 4096
    for n in (1, 13, 1000, 4096):
        x = torch.randint(0, 256, (n,), dtype=torch.uint8, device=cuda)
        for op in ("alltoall", "allgather"):
            y = torch.zeros_like(x)
            getattr(c, op)(x, y)
            torch.cuda.synchronize()
            assert torch.equal(x, y), (op, n)
        y = torch.zeros_like(x)
        c.gather(x, y, 0)
        z = torch.zeros_like(x)
        c.scatter(x, z, 0)
        torch.cuda.synchronize()
        assert torch.equal(x, y) and torch.equal(x, z), n
    big = torch.ones(8192, dtype=torch.uint8, device=cuda)  # above the cap: RCCL
    out = torch.zeros_like(big)
    before = c.peer_exchanges
    c.alltoall(big, out)
    torch.cuda.synchronize()
    assert torch.equal(big, out) and c.peer_exchanges == before
    assert c.async_error() == ""


def _run(n, *extra, timeout=110):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "-m",
           "tools.studies.peer_exchange", *extra]
    env = dict(os.environ, DTFS_SHARE_GPU="1")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, p.stdout
    return json.loads(line[0])


@pytest.mark.parametrize("n", [2, 3])
def test_peer_exchange_ranks_sharing_one_gpu(n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _run(n, "--iters", "100")
    assert out["world"] == n and out["checked_sizes"]
    for v in out["alltoall_us"].values():
        assert v["peer"] > 0 and v["rccl"] > 0


def test_peer_exchange_dead_rank_times_out():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _run(2, "--fault", "--timeout-s", "1.5")
    assert out["fault_detected"] and 1.0 <= out["waited_s"] < 20


def test_peer_exchange_falls_back_to_rccl_without_peer_access():
    """One rank reports no hipDeviceCanAccessPeer to the others: the ranks agree
    to keep every exchange on RCCL (no mailbox is mapped), and the exchanges
    stay exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = _run(2, "--deny-access", "--sizes", "1,4096")
    assert out["fallback"] == "rccl" and out["checked_sizes"] == [1, 4096]

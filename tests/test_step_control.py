"""Shared-memory step agreement (csrc/runtime/step_control.h) on its own:
proposals, per-step bucket agreement (max over ranks), bounded waits,
liveness and the sticky broken flag, across real processes."""
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.parallel.control import create_control


def _rank_main(rank, world, port, q):
    store = dist.TCPStore("127.0.0.1", port, world, rank == 0, wait_for_workers=False)
    try:
        ctl = create_control(native(), world, rank, store=store, prefix="t/ctl")
        got = []
        for k in range(20):
            if k % world == rank:
                ctl.propose(k)  # a different rank opens each step
            ctl.post(k, (k * 7 + rank * 3) % 5)
            b, err = ctl.gather(k, 10.0)
            got.append(b)
        assert ctl.proposed == 20
        store.set(f"done{rank}", "1")
        q.put((rank, got, None))
    except Exception as e:  # pragma: no cover - surfaced by the assertion
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_agreement_is_the_max_bucket_on_every_rank(world):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world):
        r, got, err = q.get(timeout=120)
        res[r] = (got, err)
    [p.join(timeout=30) for p in procs]
    want = [max((k * 7 + r * 3) % 5 for r in range(world)) for k in range(20)]
    for r in range(world):
        assert res[r][1] is None, res[r][1]
        assert res[r][0] == want


def test_timeout_liveness_and_broken_flag():
    import torch

    store = torch.distributed.HashStore()
    pfx = f"t/{os.getpid()}"
    # a 2-rank segment where rank 1 never shows up: rank 0 creates it by hand
    name = f"/dtfs-test-{os.getpid()}"
    c0 = native().StepControl(name, 2, 0, True)
    try:
        c1 = native().StepControl(name, 2, 1, False)  # attached, but never posts or beats again
        c0.propose(0)
        c0.post(0, 1)
        b, err = c0.gather(0, 0.05)
        assert b == -1 and "rank(s) 1 did not join" in err, err
        assert c0.heartbeat_age(0) < 1.0 and c0.silent_peer(10.0) == -1
        assert c0.silent_peer(0.0) == 1 or c0.heartbeat_age(1) >= 0.0
        c1.post(0, 3)
        b, err = c0.gather(0, 1.0)
        assert b == 3  # the late rank's bucket wins
        assert c0.broken_by == -1
        c1.mark_broken(1)
        assert c0.broken_by == 1 and c1.broken_by == 1
        c0.mark_broken(0)  # sticky: the first rank to give up is kept
        assert c0.broken_by == 1
        c0.propose(1)
        c0.post(1, 0)
        b, err = c0.gather(1, 5.0)  # returns at once on a broken cluster
        assert b == -1 and "broken" in err
        assert not c0.all_closing
        c0.set_closing(True)
        c1.set_closing(True)
        assert c0.all_closing and not c0.stop_requested
        c1.request_stop()
        assert c0.stop_requested and c0.epoch == 0
        c1.bump_epoch()
        assert c0.epoch == 1
        del c1
    finally:
        c0.unlink()
    with pytest.raises(RuntimeError):
        native().StepControl(name, 2, 1, False)  # unlinked: nobody can attach any more
    del store, pfx


def _attach_and_exit(name):
    from distributed_tf_serving_amd.ops import native as _native

    c = _native().StepControl(name, 2, 1, False)
    c.heartbeat()
    os._exit(0)  # no close: the segment keeps this rank's last heartbeat and pid


def test_exited_peer_is_dead_at_once():
    """A rank whose process exited is reported by silent_peer / heartbeat_age
    immediately (pid probe), not after the peer timeout: the peer exchange's
    readers stop loading from a dead owner's store within one watcher period."""
    import time
    import uuid

    name = f"/dtfs_t_{uuid.uuid4().hex[:8]}"
    c0 = native().StepControl(name, 2, 0, True)
    try:
        p = mp.get_context("spawn").Process(target=_attach_and_exit, args=(name,))
        p.start()
        p.join(timeout=60)
        assert p.exitcode == 0
        t0 = time.monotonic()
        assert c0.silent_peer(3600.0) == 1  # an hour's timeout: the pid probe decides
        assert c0.process_gone(1) and not c0.process_gone(0)
        assert c0.heartbeat_age(1) > 1e6
        assert time.monotonic() - t0 < 1.0
        for r in (-1, 2, 64):  # bounds-checked: no read past the segment's ranks
            with pytest.raises(IndexError):
                c0.process_gone(r)
    finally:
        c0.unlink()

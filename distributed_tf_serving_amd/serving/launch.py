"""Node launcher for the multi-GPU server: one process per GPU, the job's
rendezvous store in the launcher itself.

    python -m distributed_tf_serving_amd.serving.launch --nproc-per-node 8 -- \\
        -m distributed_tf_serving_amd.serving.cluster --preset deepfm_fanout4 --mode alltoall --recover

Why not ``torch.distributed.run``: its agent tears every rank down as soon as
one fails, and with a plain ``env://`` rendezvous rank 0 hosts the TCPStore,
so rank 0's death takes the store - and with it every survivor's way to agree
on a rebuilt cluster - down too. Here the launcher process, which never
touches a GPU, hosts the store (``TORCHELASTIC_USE_AGENT_STORE=True`` makes
every rank's ``init_process_group`` a store client) and lets the survivors of
a dead rank keep running; serving/cluster.py's leaderless recovery then
re-forms the cluster over them, whichever rank died (the
reference abandons a failed shard's request, DCNClient.java:185-188).

The launcher exits when every rank has exited: with 0 if every rank that was
not killed by a signal exited 0, else with the first non-zero exit code.
SIGINT / SIGTERM are forwarded to the ranks.
"""
from __future__ import annotations

import argparse
import datetime
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def start_store(host: str = "127.0.0.1", port: int = 0, timeout_s: float = 300.0):
    """A TCPStore server in this process (no GPU is touched)."""
    import torch.distributed as dist

    return dist.TCPStore(host, port, None, True, datetime.timedelta(seconds=timeout_s), wait_for_workers=False)


def rank_env(rank: int, world: int, host: str, port: int, base: Optional[dict] = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR=host, MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def launch(nproc: int, argv: Sequence[str], host: str = "127.0.0.1", port: int = 0, env: Optional[dict] = None,
           cwd: Optional[str] = None, stdout=None, stderr=None):
    """Start the store and ``nproc`` ranks running ``python <argv>``.
    Returns (store, [Popen]); the caller keeps ``store`` alive."""
    store = start_store(host, port)
    procs = [subprocess.Popen([sys.executable, *argv], env=rank_env(r, nproc, host, store.port, env), cwd=cwd,
                              stdout=stdout, stderr=stderr) for r in range(nproc)]
    return store, procs


def wait_all(procs: List[subprocess.Popen], poll_s: float = 0.2) -> int:
    while any(p.poll() is None for p in procs):
        time.sleep(poll_s)
    bad = [p.returncode for p in procs if p.returncode not in (0, None) and p.returncode > 0]
    return bad[0] if bad else 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="one process per GPU with the rendezvous store in the launcher")
    ap.add_argument("--nproc-per-node", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0, help="store port (0 = any free port)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER, help="-- <python args>, e.g. -- -m pkg.module --flag")
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd[:1] == ["--"] else a.cmd
    if not cmd:
        ap.error("nothing to launch")
    store, procs = launch(a.nproc_per_node, cmd, a.master_addr, a.master_port)

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGINT, forward)
    signal.signal(signal.SIGTERM, forward)
    rc = wait_all(procs)
    del store
    return rc


if __name__ == "__main__":
    raise SystemExit(main())

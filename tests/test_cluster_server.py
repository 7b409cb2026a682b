"""Multi-rank model server over gloo (CPU): rank 0 is the PredictionService
front door + dynamic batcher, ranks > 0 follow the step control channel; every
batch is scattered over all ranks and gathered back (reference topology:
DCNClient.java:146-164, moved inside the node)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from distributed_tf_serving_amd.config import Config, ModelConfig

    cfg = Config()
    cfg.model = ModelConfig(family="deepfm", vocab_size=5000, embed_dim=16, mlp_dims=(32, 16))
    cfg.serving.device = "cpu"
    cfg.serving.max_batch_rows = 64
    cfg.serving.allowed_batch_sizes = (16, 64)
    cfg.serving.batch_timeout_us = 500
    return cfg


def _worker(rank, world, port, q, scatter_path="shared"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.parallel.dist import init_from_env, shutdown
    from distributed_tf_serving_amd.serving.cluster import ClusterServer
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire.tensor import make_tensor_proto, to_ndarray

    try:
        ctx = init_from_env(device="cpu")
        cfg = _cfg()
        cfg.serving.scatter_path = scatter_path
        srv = ClusterServer(cfg, ctx)
        seg = srv.engine.scatter
        assert (seg is not None) == (scatter_path == "shared")
        if rank == 0:
            ref = build_model(cfg.model)
            rng = np.random.default_rng(3)
            errs = []
            for rows in (1, 7, 50, 64, 130):  # 130 > world x 64: split into several steps
                ids = rng.integers(0, 1 << 40, size=(rows, 43), dtype=np.int64)
                wts = rng.random((rows, 43), dtype=np.float32)
                req = pb.PredictRequest()
                req.model_spec.name = cfg.serving.model_name
                req.model_spec.signature_name = "serving_default"
                req.inputs["feat_ids"].CopyFrom(make_tensor_proto(ids))
                req.inputs["feat_wts"].CopyFrom(make_tensor_proto(wts))
                resp = srv.service.predict(req, timeout_s=60)
                got = to_ndarray(resp.outputs["prediction_node"])
                want = ref(torch.from_numpy(ids), torch.from_numpy(wts)).numpy()
                errs.append(float(np.abs(got - want).max()))
            stats = srv.registry.resolve(cfg.serving.model_name).scheduler.stats()
            srv.stop()
            q.put((rank, errs, (stats["steps"], stats.get("scatter_h2d_bytes", 0))))
        else:
            n = srv.serve_follower()
            srv.stop()
            q.put((rank, None, (n, seg.h2d_bytes if seg is not None else 0)))
        shutdown()
    except Exception:  # pragma: no cover - surfaced by the assertion below
        import traceback

        q.put((rank, traceback.format_exc(), -1))


@pytest.mark.parametrize("world,path", [(2, "shared"), (3, "shared"), (2, "rccl")])
def test_cluster_server_scatter_gather(world, path):
    """Scores = a local forward at every request size; every rank runs every
    step. Shared-arena scatter (csrc/runtime/shared_scatter.h): each rank
    copies only its own share of rank 0's batches (no rank copies the whole
    batch); "rccl": the collective scatter fallback (gloo here)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, path)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world):
        r, payload, steps = q.get(timeout=300)
        res[r] = (payload, steps)
    [p.join(timeout=60) for p in procs]
    errs, (steps0, _) = res[0]
    assert isinstance(errs, list), f"rank 0 failed: {errs}"
    assert max(errs) < 1e-5, errs
    for r in range(1, world):
        assert res[r][1][0] == steps0, f"rank {r} followed {res[r][1]} steps, rank 0 ran {steps0}: {res[r][0]}"
    if path == "shared":
        h2d = [res[r][1][1] for r in range(world)]
        total = sum(h2d)
        assert all(b > 0 for b in h2d), h2d
        # rank 0 copied its own share only: about 1/world of the request bytes
        # (plus 64-byte headers of steps where its share is empty)
        assert h2d[0] < total * (1.0 / world + 0.25), h2d


def _fault_worker(rank, world, port, q, die_rank, die_after):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import time

    from distributed_tf_serving_amd.parallel.dist import init_from_env
    from distributed_tf_serving_amd.serving.cluster import ClusterServer
    from distributed_tf_serving_amd.serving.errors import Code, ServingError
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire.tensor import make_tensor_proto

    try:
        ctx = init_from_env(device="cpu", timeout_s=8)
        fault = {"after": die_after} if rank == die_rank else None
        srv = ClusterServer(_cfg(), ctx, control_timeout_s=5, step_timeout_s=5, follower_fault=fault)
        if rank == 0:
            rng = np.random.default_rng(1)
            outcomes = []
            t_fail = None
            t0 = time.monotonic()
            for i in range(12):
                ids = rng.integers(0, 1 << 40, size=(40, 43), dtype=np.int64)
                wts = rng.random((40, 43), dtype=np.float32)
                req = pb.PredictRequest()
                req.model_spec.name = "DCN"
                req.inputs["feat_ids"].CopyFrom(make_tensor_proto(ids))
                req.inputs["feat_wts"].CopyFrom(make_tensor_proto(wts))
                ts = time.monotonic()
                try:
                    srv.service.predict(req, timeout_s=20)
                    outcomes.append("ok")
                except ServingError as e:
                    outcomes.append(e.code.name)
                    if t_fail is None:
                        t_fail = time.monotonic() - ts
            q.put((rank, outcomes, t_fail, srv.broken, time.monotonic() - t0))
            srv.stop()
        else:
            try:
                n = srv.serve_follower()
                q.put((rank, "stopped", n, None, 0))
            except Exception as e:  # the surviving follower: rank 0 went silent / peers gone
                q.put((rank, "raised", repr(e)[:200], None, 0))
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc(), None, None, 0))


def test_cluster_dead_follower_fails_requests_instead_of_hanging():
    """A follower dies after 2 steps: rank 0 answers the affected and every later
    request UNAVAILABLE within its step timeout (no hang), the surviving
    follower gives up on its own (reference DCNClient.java:185-188
    has no failure handling at all)."""
    world, die_rank = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, world, port, q, die_rank, 2)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world - 1):  # the dead rank reports nothing
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert 0 in res and isinstance(res[0][1], list), res
    outcomes, t_fail, broken = res[0][1], res[0][2], res[0][3]
    assert outcomes[:2] == ["ok", "ok"], outcomes
    assert "UNAVAILABLE" in outcomes and broken, (outcomes, broken)
    first_bad = outcomes.index("UNAVAILABLE")
    assert all(o == "UNAVAILABLE" for o in outcomes[first_bad:]), outcomes
    assert t_fail is not None and t_fail < 20, t_fail
    assert procs[die_rank].exitcode == 17
    assert res[1][1] in ("raised", "stopped"), res[1]


def _run_worker(n, mode, out, extra=(), env_extra=None, timeout=240):
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "tests/cluster_worker.py",
           "--mode", mode, "--out", str(out), *extra]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               DTFS_HOST_THREADS="1", **(env_extra or {}))
    return subprocess.run(cmd, cwd=repo, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("world,mode,front", [(2, "alltoall", "native"), (3, "scatter", "native"),
                                              (3, "alltoall", "grpcio")])
def test_native_cluster_serves_exact_scores_and_idles(tmp_path, world, mode, front):
    """The ClusterServer on the native live server in both fan-out modes: every
    front door's concurrent requests (raw and packed encodings, sizes that do
    not divide by the world) score exactly like a local forward, over the
    in-process service and the gRPC front door (the C++ h2c server or
    grpcio); an idle cluster launches no
    step (the step control proposes steps only for queued work)."""
    import json

    p = _run_worker(world, mode, tmp_path, ("--grpc-port", str(_free_port()), "--front", front))
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    fronts = [r for r in res if r["serves"]]
    assert len(fronts) == (world if mode == "alltoall" else 1)
    for r in fronts:
        assert r["max_diff"] < 1e-5 and r["grpc_max_diff"] < 1e-5, r
        assert r["steps_used"] < r["n_checked"]  # requests were batched
    for r in res:
        assert r["idle_steps"] == 0 and not r["broken"], r
    # every rank ran the same steps (each collective paired up)
    assert len({r["stats"]["steps"] for r in res}) == 1, [r["stats"]["steps"] for r in res]


def _recover_worker(rank, world, port, q, die_rank, die_after):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import time

    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.parallel.dist import init_from_env
    from distributed_tf_serving_amd.serving.cluster import ClusterServer
    from distributed_tf_serving_amd.serving.errors import ServingError
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire.tensor import make_tensor_proto, to_ndarray

    try:
        ctx = init_from_env(device="cpu", timeout_s=20)
        fault = {"after": die_after} if rank == die_rank else None
        cfg = _cfg()
        srv = ClusterServer(cfg, ctx, control_timeout_s=2, step_timeout_s=3, follower_fault=fault, recover=True)
        if rank == 0:
            ref = build_model(cfg.model)
            rng = np.random.default_rng(1)
            outcomes, diffs = [], []
            t_end = time.monotonic() + 90
            while time.monotonic() < t_end:
                ids = rng.integers(0, 1 << 40, size=(50, 43), dtype=np.int64)
                wts = rng.random((50, 43), dtype=np.float32)
                req = pb.PredictRequest()
                req.model_spec.name = "DCN"
                req.inputs["feat_ids"].CopyFrom(make_tensor_proto(ids))
                req.inputs["feat_wts"].CopyFrom(make_tensor_proto(wts))
                try:
                    resp = srv.service.predict(req, timeout_s=20)
                    outcomes.append("ok")
                    got = to_ndarray(resp.outputs["prediction_node"])
                    diffs.append(float(np.abs(got - ref(torch.from_numpy(ids), torch.from_numpy(wts)).numpy()).max()))
                except ServingError as e:
                    outcomes.append(e.code.name)
                    time.sleep(0.05)
                if srv.recoveries and outcomes[-5:] == ["ok"] * 5:
                    break
            q.put((rank, outcomes, diffs, srv.recoveries, srv.world))
            srv.stop()
        else:
            n = srv.serve_follower()
            q.put((rank, "stopped", n, srv.recoveries, srv.world))
            srv.stop()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc(), None, None, None))


def test_cluster_recovers_over_surviving_ranks():
    """SURVEY §5.3 degraded mode: a follower dies mid-stream; the requests in
    flight fail UNAVAILABLE, rank 0 rebuilds the cluster over the two
    survivors (fresh process group, step control and fan-out, same processes,
    same weights) and later requests are served correctly at world 2."""
    world, die_rank = 3, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_recover_worker, args=(r, world, port, q, die_rank, 3)) for r in range(world)]
    [p.start() for p in procs]
    res = {}
    for _ in range(world - 1):
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert 0 in res and isinstance(res[0][1], list), res
    outcomes, diffs, recoveries, world_after = res[0][1:]
    assert outcomes[0] == "ok" and "UNAVAILABLE" in outcomes, outcomes
    assert outcomes[-5:] == ["ok"] * 5, outcomes
    assert recoveries == 1 and world_after == 2
    assert max(diffs) < 1e-5
    assert res[1][1] == "stopped" and res[1][3] == 1 and res[1][4] == 2, res[1]
    assert procs[die_rank].exitcode == 17


def spawn_ranks(n, args, env_extra, timeout):
    """Start n worker processes directly (RANK / WORLD_SIZE / MASTER_* in the
    environment, rank 0 hosts the store): unlike torch.distributed.run's agent,
    nothing tears the survivors down when one rank dies."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_RANK=str(r), **env_extra)
        procs.append(subprocess.Popen([sys.executable, "tests/cluster_worker.py", *args], cwd=repo, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    return procs, outs


def test_cluster_worker_recovery_rehearsal_cpu(tmp_path):
    """The GPU recovery rehearsal's worker (tests/cluster_worker.py) on gloo."""
    import json

    procs, outs = spawn_ranks(3, ["--out", str(tmp_path), "--kill-rank", "2", "--kill-after", "3"],
                              dict(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
                                   DTFS_HOST_THREADS="1"), timeout=200)
    r0 = json.load(open(tmp_path / "rank0.json")) if (tmp_path / "rank0.json").exists() else None
    assert r0 is not None, [o[-2000:] for o in outs]
    assert procs[2].returncode == 17
    out = r0["outcomes"]
    assert out[0] == "ok" and "UNAVAILABLE" in out and out[-5:] == ["ok"] * 5, out
    assert r0["recoveries"] == 1 and r0["world_after"] == 2 and r0["max_diff"] < 1e-5


def spawn_launched(n, args, env_extra, timeout):
    """n ranks of tests/cluster_worker.py under serving/launch.py's model: the
    rendezvous store lives in THIS process, so any rank - rank 0 included -
    can die without taking the store with it."""
    import subprocess

    from distributed_tf_serving_amd.serving.launch import launch

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    store, procs = launch(n, ["tests/cluster_worker.py", *args], env=dict(os.environ, **env_extra), cwd=repo,
                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0].decode(errors="replace"))
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0].decode(errors="replace"))
    del store
    return procs, outs


_CPU_ENV = dict(CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", DTFS_HOST_THREADS="1")


def test_cluster_survives_rank0_death_alltoall(tmp_path):
    """Verdict r3 #7: every rank is a front door (alltoall); rank 0 - the old
    rebuild leader and store host - dies after 3 requests. The two survivors
    agree on the next epoch through the launcher-hosted store, rebuild at
    world 2 and serve exact scores again on their own front doors."""
    import json

    procs, outs = spawn_launched(3, ["--mode", "alltoall", "--out", str(tmp_path), "--kill-rank", "0",
                                     "--kill-after", "3"], _CPU_ENV, timeout=200)
    assert procs[0].returncode == 17, outs[0][-2000:]
    for r in (1, 2):
        f = tmp_path / f"rank{r}.json"
        assert f.exists(), outs[r][-3000:]
        res = json.load(open(f))
        out = res["outcomes"]
        assert out[-5:] == ["ok"] * 5, out
        assert res["recoveries"] == 1 and res["world_after"] == 2 and res["max_diff"] < 1e-5, res
        assert procs[r].returncode == 0, outs[r][-2000:]


def test_cluster_rebuilds_after_comm_error_on_idle_front_door(tmp_path):
    """an idle front door that sees a communicator error marks the
    cluster broken from Python; its own live server must go broken too (the
    watcher now honours this rank's flag), so the cluster rebuilds - here over
    all three ranks, nobody died - and serves again."""
    import json

    procs, outs = spawn_launched(3, ["--mode", "scatter", "--out", str(tmp_path), "--inject-comm-error", "0",
                                     "--kill-after", "3"], _CPU_ENV, timeout=200)
    f = tmp_path / "rank0.json"
    assert f.exists(), [o[-3000:] for o in outs]
    res = json.load(open(f))
    assert res["recoveries"] == 1 and res["world_after"] == 3, res
    assert res["outcomes"][-5:] == ["ok"] * 5 and res["max_diff"] < 1e-5, res
    for r in (1, 2):
        fr = json.load(open(tmp_path / f"rank{r}.json"))
        assert fr["recoveries"] == 1 and fr["world_after"] == 3, fr


@pytest.mark.parametrize("world", [2, 3])
def test_local_cluster_serves_sharded_dlrm_through_front_doors(tmp_path, world):
    """BASELINE config 4 as a served cluster (verdict r4 #4): every rank is a
    front door over the sharded DLRM whose tables are read where they live
    (peer exchange, no collective in the step); every request's scores - in
    process and through each rank's native gRPC door - equal the UNSHARDED
    model's; no rank idles a step; the step control carries liveness only."""
    import json

    p = _run_worker(world, "local", tmp_path, ("--preset", "dlrm", "--grpc-port", str(_free_port())))
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    assert all(r["serves"] for r in res)
    for r in res:
        assert r["max_diff"] < 1e-4 and r["grpc_max_diff"] < 1e-4, r
        assert r["idle_steps"] == 0 and not r["broken"], r
        assert r["stats"]["proposed_steps"] == 0 and r["stats"]["joined_steps"] == 0, r["stats"]  # no agreement
        # stop() ended the replica-cache refresher and the watchdog (verdict r5 #1)
        assert r["threads_after_stop"] == [], r["threads_after_stop"]
        assert "hot_cache_refreshes" in r["stats"]  # the refresher ran while serving


def test_local_cluster_dead_table_owner_unavailable_then_replanned(tmp_path):
    """SURVEY §5.3 for the peer exchange (verdict r4 #4): rank 2 - the owner of
    some tables every rank reads - dies. The survivors' watchers see its
    heartbeat stop: their requests fail UNAVAILABLE (no read of a dead
    owner's store is answered OK, nothing hangs); --recover re-plans the tables
    over the two survivors (rebuilt from their hashed initialisation) and the
    survivors serve scores equal to the unsharded model again."""
    import json

    procs, outs = spawn_launched(3, ["--mode", "local", "--preset", "dlrm", "--out", str(tmp_path), "--kill-rank",
                                     "2", "--kill-after", "3"], _CPU_ENV, timeout=240)
    assert procs[2].returncode == 17, outs[2][-2000:]
    for r in (0, 1):
        f = tmp_path / f"rank{r}.json"
        assert f.exists(), outs[r][-3000:]
        res = json.load(open(f))
        out = res["outcomes"]
        assert "UNAVAILABLE" in out and out[-5:] == ["ok"] * 5, out
        assert res["recoveries"] == 1 and res["world_after"] == 2 and res["max_diff"] < 1e-4, res
        assert procs[r].returncode == 0, outs[r][-2000:]

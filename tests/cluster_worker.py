"""One rank of a multi-rank ClusterServer rehearsal (launched by
torch.distributed.run from tests/test_cluster_server.py on CPU / gloo and from
tests/test_multirank_gpu.py on the GPU box, ranks sharing its one GPU).

Every front-door rank sends requests of assorted sizes concurrently through
the in-process PredictionService (and, with --grpc, through the gRPC front
door), compares every request's scores with a local forward of the same
weights, and checks that an idle cluster launches no steps. Each rank writes
``<out>/rank<r>.json``.
"""
import argparse
import concurrent.futures as cf
import faulthandler
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="scatter", choices=["scatter", "alltoall", "local"])
    ap.add_argument("--preset", default="deepfm", choices=["deepfm", "dlrm"],
                    help="dlrm: BASELINE config 4 scaled down - tables sharded over the ranks, read where they "
                         "live (peer exchange), checked against the unsharded model")
    ap.add_argument("--out", required=True)
    ap.add_argument("--grpc-port", type=int, default=0, help="> 0: also serve gRPC on port + rank and query it")
    ap.add_argument("--front", default="native", choices=["native", "grpcio"],
                    help="front door of the gRPC check: the C++ h2c server or grpcio")
    ap.add_argument("--requests", type=int, default=24)
    ap.add_argument("--kill-rank", type=int, default=-1, help="this rank exits abruptly after --kill-after steps")
    ap.add_argument("--kill-after", type=int, default=3)
    ap.add_argument("--inject-comm-error", type=int, default=-1,
                    help="this front-door rank reports a communicator error while idle, after --kill-after requests")
    a = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from distributed_tf_serving_amd.client.synth import SyntheticRequests
    from distributed_tf_serving_amd.config import load_preset
    from distributed_tf_serving_amd.ops import native
    from distributed_tf_serving_amd.parallel.dist import init_from_env
    from distributed_tf_serving_amd.serving.cluster import ClusterServer
    from distributed_tf_serving_amd.wire import schema as pb
    from distributed_tf_serving_amd.wire import tensor as T

    ctx = init_from_env(timeout_s=120)
    rank = ctx.rank
    gpu = ctx.device.type == "cuda"
    ref = None  # the scores every request must match (default: the served model's own forward)
    if a.preset == "dlrm":
        from distributed_tf_serving_amd.models import build_model

        cfg = load_preset("dlrm_sharded8")
        cfg.model.table_rows = 5000
        cfg.model.embedding_exchange = "peer"
        cfg.model.hot_cache_rows = 1024
        if not gpu:
            cfg.model.bottom_mlp, cfg.model.mlp_dims = (32, 64), (64, 32)
        ref = build_model(cfg.model, ctx.device)  # unsharded: the same hashed tables, materialised
    else:
        cfg = load_preset("deepfm_1gpu")
        cfg.model.vocab_size = 100_000
        if not gpu:  # small enough for gloo on a CPU test box
            cfg.model.embed_dim, cfg.model.mlp_dims = 16, (32, 16)
    cfg.serving.model_name = "DCN"
    cfg.serving.device = "cuda" if gpu else "cpu"
    cfg.serving.max_batch_rows = 768
    cfg.serving.allowed_batch_sizes = (96, 768)  # divisible by 1, 2, 3
    cfg.serving.batch_timeout_us = 300
    phase = dist.new_group(backend="gloo")
    fault = {"after": a.kill_after} if rank == a.kill_rank and a.mode == "scatter" else None
    if a.kill_rank >= 0 or a.inject_comm_error >= 0:
        # recovery rehearsal: rank a.kill_rank dies after a few steps (a scatter
        # follower by its step count, an alltoall front door after kill_after of
        # its own requests - rank 0 included), or rank a.inject_comm_error (an
        # idle front door) reports a communicator error; every front door keeps
        # sending requests until the rebuilt cluster served 5 in a row
        srv = ClusterServer(cfg, ctx, mode=a.mode, control_timeout_s=3, step_timeout_s=5, follower_fault=fault,
                            recover=True)
        res = {"rank": rank}
        if srv.serves:
            from distributed_tf_serving_amd.serving.errors import ServingError

            model = ref or srv.registry.resolve("DCN").model
            synth = SyntheticRequests(fields=43, id_space=1 << 40, dist="zipf", seed=7 + rank)
            outcomes, diffs = [], []
            t_end = time.monotonic() + 70
            injected = False
            while time.monotonic() < t_end:
                n_ok = outcomes.count("ok")
                if a.mode in ("alltoall", "local") and rank == a.kill_rank and n_ok >= a.kill_after:
                    os._exit(17)
                if rank == a.inject_comm_error and n_ok >= a.kill_after and not injected:
                    time.sleep(0.3)  # the front door is idle when the error arrives
                    srv.inject_comm_error()
                    injected = True
                ids, wts = synth.arrays(300)
                data = native().encode_predict_request("DCN", "serving_default", None,
                                                       [("feat_ids", torch.from_numpy(ids)),
                                                        ("feat_wts", torch.from_numpy(wts))], True)
                try:
                    resp = srv.service.predict_bytes(data, 30.0)
                    got = T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])
                    want = model(torch.from_numpy(ids).to(ctx.device), torch.from_numpy(wts).to(ctx.device))
                    diffs.append(float(np.abs(got - want.float().cpu().numpy()).max()))
                    outcomes.append("ok")
                except ServingError as e:
                    outcomes.append(e.code.name)
                    time.sleep(0.05)
                if srv.recoveries and outcomes[-5:] == ["ok"] * 5:
                    break
            res.update(outcomes=outcomes, max_diff=max(diffs) if diffs else None, recoveries=srv.recoveries,
                       world_after=srv.world)
            with open(os.path.join(a.out, f"rank{rank}.json"), "w") as f:
                json.dump(res, f)  # before stop(): a survivor's peers may already be gone
            # alltoall / local: every front door keeps its live server up (joining
            # the others' steps; local: its table shards stay mapped by the
            # others) until all of this epoch's front doors are done
            key = f"test/done/{srv.epoch}"
            srv._store.add(key, 1)
            t_wait = time.monotonic() + 60
            while srv.mode in ("alltoall", "local") and srv._store.add(key, 0) < srv.world and \
                    time.monotonic() < t_wait:
                time.sleep(0.05)
            srv.stop()
        else:
            res["followed"] = srv.serve_follower()
            res.update(recoveries=srv.recoveries, world_after=srv.world)
            srv.stop()
            with open(os.path.join(a.out, f"rank{rank}.json"), "w") as f:
                json.dump(res, f)
        return
    srv = ClusterServer(cfg, ctx, mode=a.mode, control_timeout_s=20, step_timeout_s=20, follower_fault=fault)
    res = {"rank": rank, "serves": srv.serves}
    if srv.serves:
        model = ref or srv.registry.resolve("DCN").model
        synth = SyntheticRequests(fields=43, id_space=1 << 40, dist="zipf", seed=100 + rank)
        reqs = []
        for i in range(a.requests):
            rows = [1, 37, 200, 96, 500, 7][i % 6]
            ids, wts = synth.arrays(rows)
            raw = i % 3 != 2  # raw tensor_content and packed typed fields
            data = native().encode_predict_request("DCN", "serving_default", None,
                                                   [("feat_ids", torch.from_numpy(ids)),
                                                    ("feat_wts", torch.from_numpy(wts))], raw)
            reqs.append((data, ids, wts))
        steps0 = srv.sched.stats()["steps"]
        with cf.ThreadPoolExecutor(8) as pool:
            outs = list(pool.map(lambda r: srv.service.predict_bytes(r[0], 60.0), reqs))
        diffs = []
        for (data, ids, wts), resp in zip(reqs, outs):
            got = T.to_ndarray(pb.PredictResponse.FromString(resp).outputs["prediction_node"])
            want = model(torch.from_numpy(ids).to(ctx.device), torch.from_numpy(wts).to(ctx.device)).float().cpu()
            diffs.append(float(np.abs(got - want.numpy()).max()))
        res["max_diff"] = max(diffs)
        res["n_checked"] = len(diffs)
        res["steps_used"] = srv.sched.stats()["steps"] - steps0
        if a.grpc_port:
            from distributed_tf_serving_amd.client.backends import GrpcBackend

            # alltoall: every rank is a front door; an ephemeral port each (port + rank
            # could collide with the rendezvous / RCCL sockets)
            p = 0 if a.mode in ("alltoall", "local") else a.grpc_port
            port = (srv.start_native_grpc(p, host="127.0.0.1") if a.front == "native"
                    else srv.start_grpc(p, host="127.0.0.1"))
            be = GrpcBackend(f"127.0.0.1:{port}")
            gd = []
            for data, ids, wts in reqs[:4]:
                resp = pb.PredictResponse.FromString(be.predict(data, timeout_s=60.0))
                got = T.to_ndarray(resp.outputs["prediction_node"])
                want = model(torch.from_numpy(ids).to(ctx.device), torch.from_numpy(wts).to(ctx.device)).float().cpu()
                gd.append(float(np.abs(got - want.numpy()).max()))
            be.close()
            res["grpc_max_diff"] = max(gd)
    dist.barrier(group=phase)  # every front door is done: the cluster is idle now
    # let the last step's bookkeeping land (a rank that joined a peer's final
    # step may count it a moment after that peer's front door answered; under
    # a loaded CPU that moment can exceed the window below)
    st0 = srv.sched.stats()["steps"]
    for _ in range(40):
        time.sleep(0.05)
        st1 = srv.sched.stats()["steps"]
        if st1 == st0:
            break
        st0 = st1
    time.sleep(0.3)
    res["idle_steps"] = srv.sched.stats()["steps"] - st0
    res["stats"] = {k: v for k, v in srv.sched.stats().items() if isinstance(v, (int, float))}
    dist.barrier(group=phase)
    if srv.serves:
        srv.stop()
    else:
        res["followed"] = srv.serve_follower()
        srv.stop()
    res["broken"] = bool(srv.broken)
    # stop() joins the watchdog and the replica-cache refresher: nothing of the
    # server may still run (and touch peer memory) while the process exits
    res["threads_after_stop"] = [t.name for t in threading.enumerate() if t.name.startswith("dtfs-")]
    with open(os.path.join(a.out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier(group=phase)


if __name__ == "__main__":
    _out = next((sys.argv[i + 1] for i, x in enumerate(sys.argv[:-1]) if x == "--out"), None)
    # a native abort (SIGABRT / SIGSEGV) still names the Python frame of every
    # thread: into rank<r>.fault, where the test reads it (torchrun's failure
    # summary keeps only the signal)
    _fault = open(os.path.join(_out, f"rank{os.environ.get('RANK', '?')}.fault"), "w") if _out else sys.stderr
    faulthandler.enable(file=_fault, all_threads=True)
    try:
        main()
    except BaseException:
        # torchrun's failure summary hides a rank's own traceback: leave it where the test looks
        import traceback

        out = next((sys.argv[i + 1] for i, x in enumerate(sys.argv[:-1]) if x == "--out"), None)
        if out:
            with open(os.path.join(out, f"rank{os.environ.get('RANK', '?')}.err"), "w") as f:
                f.write(traceback.format_exc())
        raise

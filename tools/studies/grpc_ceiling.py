"""Where does the gRPC front door top out? (VERDICT r1 "What's weak" 1)

Starts ``serving.server`` (gRPC PredictionService over the native live server)
in a child process, then drives it with P client PROCESSES x T threads of
blocking unary Predict calls carrying pre-serialized requests (identity
serializers: no client-side protobuf work), closed loop, for D seconds per
point. For each P it reports the achieved RPC/s, scores/s, latency
percentiles, and the server process's CPU use (psutil) - enough to tell a
client-bound curve (rate grows with P) from a server-bound one (flat rate,
server CPU pinned), and the live server's own batching stats through the
Prometheus endpoint.

    python -m tools.studies.grpc_ceiling --preset deepfm_1gpu --procs 1 2 4
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

METHOD = "/tensorflow.serving.PredictionService/Predict"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _client_proc(port, threads, seconds, rows, raw, seed, q):
    import threading

    import grpc

    from distributed_tf_serving_amd.client.synth import SyntheticRequests

    synth = SyntheticRequests(fields=43, id_space=1 << 40, dist="zipf", seed=seed)
    reqs = [synth.serialized(rows, raw=raw) for _ in range(16)]
    opts = [("grpc.max_receive_message_length", 64 << 20), ("grpc.max_send_message_length", 64 << 20)]
    chans = [grpc.insecure_channel(f"127.0.0.1:{port}", options=opts) for _ in range(max(1, threads // 8))]
    calls = [c.unary_unary(METHOD, request_serializer=lambda b: b, response_deserializer=lambda b: b) for c in chans]
    lat, errs = [], [0]
    lock = threading.Lock()
    t_end = time.monotonic() + seconds

    def run(k):
        call = calls[k % len(calls)]
        mine = []
        i = k
        while time.monotonic() < t_end:
            t0 = time.perf_counter()
            try:
                call(reqs[i % len(reqs)], timeout=30)
                mine.append((time.perf_counter() - t0) * 1e3)
            except grpc.RpcError:
                with lock:
                    errs[0] += 1
            i += 1
        with lock:
            lat.extend(mine)

    ts = [threading.Thread(target=run, args=(k,)) for k in range(threads)]
    t0 = time.monotonic()
    [t.start() for t in ts]
    [t.join() for t in ts]
    q.put((lat, errs[0], time.monotonic() - t0))


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--preset", default="deepfm_1gpu")
    ap.add_argument("--procs", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--packed", action="store_true", help="int64_val/float_val (the reference client's encoding)")
    ap.add_argument("--grpc-workers", type=int, default=64)
    ap.add_argument("--frontends", type=int, default=1, help="server processes sharing the port")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    import psutil

    port, mport = _free_port(), _free_port()
    env = dict(os.environ)
    srv = subprocess.Popen([sys.executable, "-u", "-m", "distributed_tf_serving_amd.serving.server", "--preset",
                            a.preset, "--port", str(port), "--grpc-workers", str(a.grpc_workers),
                            "--monitoring-port", str(mport), "--frontends", str(a.frontends)], env=env,
                           stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True)
    try:
        t0 = time.time()
        while True:
            line = srv.stdout.readline()
            if "serving model" in line:
                break
            if srv.poll() is not None or time.time() - t0 > 240:
                raise RuntimeError(f"server did not start: {line}")
        time.sleep(3.0 * (a.frontends - 1))  # the other frontends finish their start-up
        sp = psutil.Process(srv.pid)
        results = []
        ctx = mp.get_context("spawn")
        for P in a.procs:
            q = ctx.Queue()
            ps = [ctx.Process(target=_client_proc, args=(port, a.threads, a.seconds, a.rows, not a.packed, 7 + k, q))
                  for k in range(P)]
            [p.start() for p in ps]
            time.sleep(min(2.0, a.seconds / 3))  # clients warm up; then sample the server
            procs = [sp] + sp.children(recursive=True)

            def cpu():
                t = 0.0
                for pr in procs:
                    try:
                        c = pr.cpu_times()
                        t += c.user + c.system
                    except psutil.Error:
                        pass
                return t

            c0 = cpu()
            w0 = time.monotonic()
            outs = [q.get(timeout=a.seconds + 120) for _ in ps]
            c1 = cpu()
            w1 = time.monotonic()
            [p.join(timeout=30) for p in ps]
            lat = np.concatenate([np.asarray(o[0]) for o in outs]) if outs else np.zeros(0)
            wall = max(o[2] for o in outs)
            n = len(lat)
            cpu_cores = (c1 - c0) / max(1e-9, w1 - w0)
            r = {"client_procs": P, "threads_per_proc": a.threads, "rpcs": int(n),
                 "errors": int(sum(o[1] for o in outs)), "rpc_per_s": round(n / wall, 1),
                 "scores_per_s": round(n * a.rows / wall, 1),
                 "p50_ms": round(float(np.percentile(lat, 50)), 3) if n else None,
                 "p99_ms": round(float(np.percentile(lat, 99)), 3) if n else None,
                 "server_cpu_cores": round(cpu_cores, 2), "server_threads": sp.num_threads(),
                 "frontends": a.frontends}
            print(json.dumps(r), flush=True)
            results.append(r)
        try:
            import urllib.request

            metrics = urllib.request.urlopen(f"http://127.0.0.1:{mport}/metrics", timeout=5).read().decode()
            keep = [ln for ln in metrics.splitlines() if "batching" in ln and not ln.startswith("#")]
        except Exception as e:  # noqa: BLE001
            keep = [f"metrics unavailable: {e}"]
        out = {"preset": a.preset, "rows": a.rows, "encoding": "packed" if a.packed else "raw",
               "frontends": a.frontends,
               "grpc_workers": a.grpc_workers, "points": results, "server_batching_metrics": keep}
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        srv.send_signal(signal.SIGINT)
        try:
            srv.wait(timeout=30)
        except subprocess.TimeoutExpired:
            srv.kill()


if __name__ == "__main__":
    main()

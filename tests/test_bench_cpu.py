"""bench.py contract on CPU: the driver's launch line (torch.distributed.run,
one rank per device, 127.0.0.1 rendezvous) with gloo, world sizes 1 and 2,
tiny step shapes. Checks the single JSON line the driver parses (whole-job
value, n_gpus, steps/warmup, weak scaling, global batch = N x per-rank rows).

Round 3 saw an intermittent SIGSEGV of the world-1 run here (2 of ~10
full-suite runs). Root cause: the native load generator's completion
callback touched run_load's stack after the waiter could return
(csrc/runtime/loadgen.cpp, use-after-return); fixed, with a deterministic
regression test in tests/test_live_server.py, and these suites now run
clean under ASan with detect_stack_use_after_return (scripts/sanitize_native.sh)."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_bench(n: int, extra=()):
    args = ["bench.py", "--gpus", str(n), "--steps", "2", "--warmup", "1", "--prime-steps", "0", "--requests-per-gpu", "1",
            "--request-rows", "64", "--pool", "2", "--client-threads", "2", *extra]
    if n == 1:
        cmd = [sys.executable, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               DTFS_HOST_THREADS="1", DTFS_HANG_DUMP_S="240")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only, one line
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2])
def test_bench_json_contract(n):
    out = _run_bench(n)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["dtype"] == "bf16" and "synthetic" in out["data"]
    assert out["config"]["global_batch"] == n * 64
    assert out["value"] > 0
    # value is the whole-job rate: global rows per step / seconds per step
    assert out["value"] == pytest.approx(n * 64 / (out["ms_per_step"] * 1e-3), rel=0.02)
    assert f"candidate-dp{n}" in out["config"]["parallelism"]


def test_bench_scatter_mode_world2():
    out = _run_bench(2, ("--mode", "scatter"))
    assert "scatter" in out["config"]["parallelism"] and out["config"]["global_batch"] == 128
    # shared-arena scatter: each rank copied its own share of rank 0's batches
    per = out["scatter"]["h2d_bytes_per_step_by_rank"]
    assert len(per) == 2 and all(b > 64 for b in per), per


def test_bench_scatter_mode_rccl_path_world2():
    out = _run_bench(2, ("--mode", "scatter", "--scatter-path", "rccl"))
    assert "scatter" in out["config"]["parallelism"] and "scatter" not in out


@pytest.mark.slow
@pytest.mark.parametrize("n,mode", [(4, "alltoall"), (8, "alltoall"), (4, "scatter"), (8, "scatter"), (4, "local")])
def test_bench_more_ranks(n, mode):
    """World 4 and 8 over gloo, with requests (20 rows) that do not divide by
    the world size: every rank must finish the same lockstep steps (no hang)
    and the job reports the whole-node rate."""
    out = _run_bench(n, ("--mode", mode, "--request-rows", "20", "--requests-per-gpu", "2"))
    assert out["n_gpus"] == n and out["config"]["global_batch"] == n * 40
    assert out["value"] == pytest.approx(n * 40 / (out["ms_per_step"] * 1e-3), rel=0.02)
    assert out.get("requests_failed", 0) == 0
    assert (mode in out["config"]["parallelism"]) or (mode == "local" and "replica" in out["config"]["parallelism"])


@pytest.mark.slow
@pytest.mark.parametrize("n,model", [(8, "dcn_v2"), (3, "dcn_v2"), (8, "deepfm")])
def test_bench_alltoall_fanout_exact_vs_local(n, model):
    """BASELINE config 5 (DCN-v2, fp8 towers) and config 3 (DeepFM) fanned out
    over n gloo ranks in alltoall mode (every rank a front door, its rows split
    over all ranks as narrow exchange rows): at start-up every bucket's fan-out
    step scores exactly like a local forward of the same rows on every rank,
    and the served run fails no request."""
    out = _run_bench(n, ("--model", model, "--mode", "alltoall", "--request-rows", "24", "--requests-per-gpu", "2",
                         "--small-buckets", "", "--qps", "0", "--qps-sweep", ""))
    assert out["n_gpus"] == n and out.get("requests_failed", 0) == 0
    assert "alltoall" in out["config"]["parallelism"], out["config"]["parallelism"]
    sc = out["self_check"]
    assert sc["buckets"] and all(b["max_abs_diff"] <= 1e-5 and b["rows"] > 0 for b in sc["buckets"]), sc


@pytest.mark.slow
def test_bench_sharded_dlrm_world2():
    """DLRM with tables sharded over 2 gloo ranks: every step is the eager step
    program (ids all-to-all, owner gather, embeddings all-to-all) in lockstep."""
    out = _run_bench(2, ("--model", "dlrm", "--table-rows", "5000"))
    par = out["config"]["parallelism"]
    assert "embedding-mp2" in par and "candidate-dp2" in par, par
    assert out.get("requests_failed", 0) == 0 and out["config"]["global_batch"] == 128


@pytest.mark.slow
def test_bench_sharded_dlrm_peer_exchange_world2():
    """--exchange peer: each rank loads remote rows from its peer's store (a
    shared-memory file on the CPU), the hot-row replica cache fills from the
    kernels' samples before the clock starts, and the JSON reports its hit
    rate and the bytes that crossed to the peer per step."""
    out = _run_bench(2, ("--model", "dlrm", "--table-rows", "5000", "--exchange", "peer", "--hot-cache-rows", "4096",
                         "--cache-learn-rounds", "2", "--cache-learn-requests", "16"))
    par = out["config"]["parallelism"]
    assert "embedding-mp2" in par and "xGMI" in par and "replica cache" in par, par
    ex = out["embedding_exchange"]
    assert ex["mode"] == "peer" and ex["hot_row_cache"] is not None
    c = ex["hot_row_cache"]
    assert c["hot_rows"] > 0 and c["refreshes"] >= 2 and c["remote_lookups_per_step"] > 0
    # the exact top-k of the served pool's keys bounds what any hot set of k rows can hit
    o = c["oracle"]
    assert o["distinct_keys"] > 0 and 0 < o["hit_rate_at"][str(c["capacity_rows"])] <= 1.0, o
    assert 0.0 < c["hit_rate"] <= 1.0 and 0.0 <= c["hit_rate_fresh_stream"] <= 1.0
    assert c["xgmi_bytes_per_step_per_rank"] < ex["bytes_per_step_per_rank"]
    assert out.get("requests_failed", 0) == 0


@pytest.mark.slow
def test_bench_sharded_dlrm_peer_exchange_world8():
    """The 8-rank shape of config 4 rehearsed over gloo: 26 tables placed on 8
    ranks, every rank loading from 7 peers' stores, caches sized automatically
    (capped at the remote rows), whole-job rate over 8 ranks."""
    out = _run_bench(8, ("--model", "dlrm", "--table-rows", "2000", "--exchange", "peer", "--cache-learn-rounds", "1",
                         "--cache-learn-requests", "8", "--stream-pool", "64",
                         "--request-rows", "20", "--requests-per-gpu", "2"))
    par = out["config"]["parallelism"]
    assert "embedding-mp8" in par and out["n_gpus"] == 8 and out["config"]["global_batch"] == 8 * 40, par
    c = out["embedding_exchange"]["hot_row_cache"]
    assert c is not None and c["sized"].startswith("auto") and c["capacity_rows"] > 0
    assert out.get("requests_failed", 0) == 0


@pytest.mark.parametrize("n", [1, 2])
def test_bench_reference_workload(n):
    """--reference-workload: the reference's closed loop (DCN, 1500 identical
    candidates, 6 clients) prints the reference's average line; at N = 2 rank
    0 scatters every request over both ranks."""
    args = ["bench.py", "--gpus", str(n), "--reference-workload", "--ref-requests", "2", "--decode-threads", "1"]
    cmd = [sys.executable, *args] if n == 1 else [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               DTFS_HOST_THREADS="1", DTFS_HANG_DUMP_S="240")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert "Average time cost with 1500 is " in p.stdout and " ms with 12 requests" in p.stdout, p.stdout
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["errors"] == 0 and out["requests"] == 12 and out["n_gpus"] == n


def test_bench_reference_workload_over_grpc():
    """--reference-workload --over-grpc: the clients are a separate process of
    native h2c gRPC clients against the native gRPC front door over TCP."""
    args = ["bench.py", "--reference-workload", "--over-grpc", "--ref-requests", "3", "--decode-threads", "1",
            "--grpc-threads", "2"]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1",
               DTFS_HOST_THREADS="1", DTFS_HANG_DUMP_S="240")
    p = subprocess.run([sys.executable, *args], cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    assert "Average time cost with 1500 is " in p.stdout and " ms with 18 requests" in p.stdout, p.stdout
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert out["errors"] == 0 and out["requests"] == 18 and out["front_door"]["protocol_errors"] == 0, out
    assert out["requests_per_s"] > 0 and "native gRPC front door" in out["path"]


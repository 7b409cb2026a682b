"""Where the ~13 us idle between two served DeepFM steps comes from: the
one-launch tower (ops.gather_mlp) back to back on one stream, with the pieces
of a served step added one at a time (interleaved rounds, per-launch period):

  plain      device output, nothing between launches
  pinned     scores written straight to pinned host memory (the served form)
  wait_done  + a wait on an event of another stream that has long completed
  wait_h2d   + a 5 MB pinned H2D per launch on a copy stream, waited on (the served step)
  h2d_nowait the same copies, not waited on (their traffic alone)
  d2d_nowait 5 MB device-to-device copies on the copy stream instead, not waited on
  wait_fresh a wait on an event recorded on the copy stream each launch, no copy
  flag_h2d   the served copies, waited on through a 32-bit flag (hipStreamWriteValue32 after the copy,
             hipStreamWaitValue32 before the tower) instead of an event
  host_fed   the served copies issued ahead by a second host thread; each tower is enqueued once the
             host sees its copy's event complete (no cross-queue wait packet on the compute queue)

    python -m tools.studies.step_gap_study [--rows 16384]
"""
from __future__ import annotations

import argparse
import json
import statistics
import threading
import time

import torch

from distributed_tf_serving_amd import ops
from distributed_tf_serving_amd.ops import hip
from distributed_tf_serving_amd.client.synth import SyntheticRequests
from distributed_tf_serving_amd.config import ModelConfig
from distributed_tf_serving_amd.models import build_model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = build_model(ModelConfig(family="deepfm", vocab_size=1_000_000), dev)
    B = a.rows
    ids, wts = SyntheticRequests(fields=43, id_space=1 << 40, dist="zipf", seed=B).arrays(B)
    ids, wts = torch.from_numpy(ids).to(dev), torch.from_numpy(wts).to(dev)
    out_d = torch.empty(B, dtype=torch.float32, device=dev)
    out_h = torch.empty(B, dtype=torch.float32, pin_memory=True)
    src = torch.empty(5 << 20, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(5 << 20, dtype=torch.uint8, device=dev)
    dst2 = torch.empty(5 << 20, dtype=torch.uint8, device=dev)
    bufs = [torch.empty(5 << 20, dtype=torch.uint8, device=dev) for _ in range(4)]
    comp, copy = torch.cuda.Stream(), torch.cuda.Stream()
    done_ev = torch.cuda.Event()
    with torch.cuda.stream(copy):
        done_ev.record()
    torch.cuda.synchronize()

    def tower(out):
        ops.gather_mlp(m.emb, ids, wts, m.lin, m.cfg.vocab_size, m.fm_bias, m.mlp.layers, m.head_w, m.head_b,
                       fm=True, out=out)

    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    seq = [0]

    def run(variant):
        base = seq[0]
        seq[0] += a.iters
        evs = [torch.cuda.Event() for _ in range(a.iters)]
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        issued = [threading.Event() for _ in range(a.iters)]

        def copier():  # host_fed: copies issued ahead, each on its own buffer slot (4 in flight at most)
            with torch.cuda.stream(copy):
                for i in range(a.iters):
                    if i >= 4:
                        issued[i - 4].wait()
                        while not towers_done[i - 4].query():
                            time.sleep(0)
                    bufs[i % 4].copy_(src, non_blocking=True)
                    evs[i].record(copy)
                    issued[i].set()

        towers_done = [torch.cuda.Event() for _ in range(a.iters)]
        with torch.cuda.stream(comp):
            tower(out_d)
            torch.cuda.synchronize()
            s.record(comp)
            if variant == "host_fed":
                th = threading.Thread(target=copier)
                th.start()
                for i in range(a.iters):
                    issued[i].wait()
                    while not evs[i].query():
                        time.sleep(0)
                    tower(out_h)
                    towers_done[i].record(comp)
                th.join()
            for i in range(a.iters if variant != "host_fed" else 0):
                if variant == "wait_done":
                    comp.wait_event(done_ev)
                elif variant == "wait_fresh":
                    evs[i].record(copy)
                    comp.wait_event(evs[i])
                elif variant == "flag_h2d":
                    with torch.cuda.stream(copy):
                        dst.copy_(src, non_blocking=True)
                    hip().stream_write_u32(copy.cuda_stream, flag, base + i + 1)
                    hip().stream_wait_u32(comp.cuda_stream, flag, base + i + 1)
                elif variant in ("wait_h2d", "h2d_nowait", "d2d_nowait"):
                    with torch.cuda.stream(copy):
                        dst.copy_(dst2 if variant == "d2d_nowait" else src, non_blocking=True)
                        evs[i].record(copy)
                    if variant == "wait_h2d":
                        comp.wait_event(evs[i])
                tower(out_d if variant == "plain" else out_h)
            e.record(comp)
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / a.iters

    variants = ["plain", "pinned", "wait_done", "wait_h2d", "h2d_nowait", "d2d_nowait", "wait_fresh", "flag_h2d", "host_fed"]
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            times[v].append(run(v))
    print(json.dumps({"rows": B, **{f"{v}_us": round(statistics.median(t), 2) for v, t in times.items()}}), flush=True)


if __name__ == "__main__":
    main()

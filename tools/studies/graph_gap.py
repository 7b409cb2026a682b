"""Where does the time between two serving steps go? (run under rocprofv3)

    rocprofv3 --kernel-trace -d out -o run -- python3 -m tools.studies.graph_gap
    python -m tools.studies.graph_gap --analyze out/run_results.db

Phases (separated by 20 ms idle gaps in the trace):
  A  the DeepFM step graph replayed back-to-back on one stream
  B  the same, each replay behind a wait on an event of another stream
  C  the same forward launched eagerly (no graph)
  D  the same forward replayed from a second graph captured per slot, slots
     alternating (what the serving loop does)
For each phase: median idle time between the last kernel of step k and the
first kernel of step k+1.
"""
from __future__ import annotations

import argparse
import statistics
import time


def run(B: int = 8192, iters: int = 30):
    import torch

    from distributed_tf_serving_amd.config import ModelConfig
    from distributed_tf_serving_amd.models import build_model
    from distributed_tf_serving_amd.serving.executor import ShardExecutor
    from distributed_tf_serving_amd.serving.packing import PackedLayout

    dev = torch.device("cuda", 0)
    cfg = ModelConfig(family="deepfm")
    m = build_model(cfg, dev)
    L = PackedLayout(cfg.num_fields)
    ex = ShardExecutor(m, L, [B], dev, slots=2)
    for s in range(2):
        buf = ex.input_buffer(B, s)
        L.ids(buf).copy_(torch.randint(0, 1 << 40, (B, cfg.num_fields), device=dev))
        L.wts(buf).copy_(torch.rand(B, cfg.num_fields, device=dev))
        ex.prepare(B, s)
    g0 = ex._graphs[(B, 0)]
    g1 = ex._graphs[(B, 1)]
    cur = torch.cuda.current_stream(dev)
    other = torch.cuda.Stream(dev)

    def idle():
        torch.cuda.synchronize()
        time.sleep(0.02)

    idle()
    for _ in range(iters):  # A
        g0.replay()
    idle()
    for _ in range(iters):  # B
        ev = torch.cuda.Event()
        with torch.cuda.stream(other):
            ev.record(other)
        cur.wait_event(ev)
        g0.replay()
    idle()
    buf = ex.input_buffer(B, 0)
    for _ in range(iters):  # C
        ex._forward(buf)
    idle()
    for i in range(iters):  # D
        (g0 if i % 2 == 0 else g1).replay()
    idle()


def analyze(db: str, first: str = "unpack|embed", last: str = "gemm_head"):
    import re
    import sqlite3

    c = sqlite3.connect(db)
    rows = [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    phases, cur = [], []
    for r in rows:
        if cur and r[1] - cur[-1][2] > 10_000_000:  # 10 ms idle: next phase
            phases.append(cur)
            cur = []
        cur.append(r)
    if cur:
        phases.append(cur)
    fr, lr = re.compile(first), re.compile(last)
    for i, ph in enumerate(phases):
        gaps, spans = [], []
        for a, b in zip(ph, ph[1:]):
            if lr.search(a[0]) and fr.search(b[0]):
                gaps.append((b[1] - a[2]) / 1e3)
        starts = [r[1] for r in ph if fr.search(r[0])]
        if len(starts) > 2:
            spans = [(b - a) / 1e3 for a, b in zip(starts, starts[1:])]
        if gaps:
            print(f"phase {i}: {len(ph)} kernels, step period median {statistics.median(spans):.1f} us, "
                  f"gap last->first median {statistics.median(gaps):.1f} us (min {min(gaps):.1f})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default="")
    ap.add_argument("--batch", type=int, default=8192)
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.batch)


if __name__ == "__main__":
    main()

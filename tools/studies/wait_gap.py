"""What does a cross-stream dependency cost on the compute queue? (run under rocprofv3)

    rocprofv3 --kernel-trace -d out -o run -- python3 -m tools.studies.wait_gap
    python -m tools.studies.wait_gap --analyze out/run_results.db

The serving step waits for its H2D copy (copy stream) before its first
kernel. The trace showed a ~10 us idle gap at exactly that point every step
even though the copy had finished long before. Phases (separated by 20 ms
idle gaps), each a chain of identical GEMM kernels on one stream:
  0  no dependency                                     (floor)
  1  hipStreamWaitEvent on an event of another stream that completed long ago
  2  the same with an H2D copy per step on the copy stream (the serving shape)
  3  hipStreamWaitValue32 on a device flag the copy stream wrote long ago
  4  the wait skipped when hipEventQuery says the event already completed
  5  an event recorded on the compute stream after every kernel (no waits)
  6  5 + the host synchronizes on the event of two kernels back (serving loop)
  7  6 + the completed cross-stream wait before each kernel
  8  the serving loop's shape with a small (64 KB) copy: copy stream waits
     done[k-4], copies, records; compute waits it, runs, records done[k];
     the host synchronizes on done[k-2]
Printed: median idle time between consecutive kernels per phase.
"""
from __future__ import annotations

import argparse
import ctypes
import statistics
import time


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32]
    lib.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    lib.hipEventQuery.argtypes = [ctypes.c_void_p]
    return lib


def run(iters: int = 40):
    import torch

    dev = torch.device("cuda", 0)
    hip = _hip()
    a = torch.randn(8192, 2752, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2752, 1024, device=dev, dtype=torch.bfloat16)
    out = torch.empty(8192, 1024, device=dev, dtype=torch.bfloat16)
    host = torch.empty(8 << 20, dtype=torch.uint8).pin_memory()
    dbuf = torch.empty(8 << 20, dtype=torch.uint8, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    cur = torch.cuda.current_stream(dev)
    other = torch.cuda.Stream(dev)
    GE, EQ = 3, 0  # hipStreamWaitValueGte, ...

    def work():
        torch.mm(a, w, out=out)

    def idle():
        torch.cuda.synchronize()
        time.sleep(0.02)

    for _ in range(5):
        work()
    idle()
    for _ in range(iters):  # 0
        work()
    idle()
    evs = []
    for _ in range(iters):
        ev = torch.cuda.Event()
        ev.record(other)
        evs.append(ev)
    torch.cuda.synchronize()
    for ev in evs:  # 1
        cur.wait_event(ev)
        work()
    idle()
    for _ in range(iters):  # 2
        with torch.cuda.stream(other):
            dbuf.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(other)
        cur.wait_event(ev)
        work()
    idle()
    hip.hipStreamWriteValue32(ctypes.c_void_p(other.cuda_stream), ctypes.c_void_p(flag.data_ptr()), 7, 0)
    torch.cuda.synchronize()
    for _ in range(iters):  # 3
        hip.hipStreamWaitValue32(ctypes.c_void_p(cur.cuda_stream), ctypes.c_void_p(flag.data_ptr()), 7, GE,
                                 0xFFFFFFFF)
        work()
    idle()
    for ev in evs:  # 4
        if not ev.query():
            cur.wait_event(ev)
        work()
    idle()
    for _ in range(iters):  # 5
        work()
        torch.cuda.Event().record(cur)
    idle()
    done = []
    for i in range(iters):  # 6
        work()
        ev = torch.cuda.Event()
        ev.record(cur)
        done.append(ev)
        if i >= 2:
            done[i - 2].synchronize()
    idle()
    done = []
    for i, ev0 in enumerate(evs):  # 7
        cur.wait_event(ev0)
        work()
        ev = torch.cuda.Event()
        ev.record(cur)
        done.append(ev)
        if i >= 2:
            done[i - 2].synchronize()
    idle()
    done = []
    small_h, small_d = host[: 64 << 10], dbuf[: 64 << 10]
    for i in range(iters):  # 8
        with torch.cuda.stream(other):
            if i >= 4:
                other.wait_event(done[i - 4])
            small_d.copy_(small_h, non_blocking=True)
            h2d = torch.cuda.Event()
            h2d.record(other)
        cur.wait_event(h2d)
        work()
        ev = torch.cuda.Event()
        ev.record(cur)
        done.append(ev)
        if i >= 2:
            done[i - 2].synchronize()
    idle()


def analyze(db: str):
    import sqlite3

    c = sqlite3.connect(db)
    rows = [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    phases, cur = [], []
    for r in rows:
        if cur and r[1] - cur[-1][2] > 10_000_000:
            phases.append(cur)
            cur = []
        cur.append(r)
    if cur:
        phases.append(cur)
    names = ["no dependency", "event wait (completed)", "event wait (H2D per step)", "wait-value (set)",
             "wait skipped if complete", "record after each", "record + host sync k-2", "wait + record + sync",
             "serving-loop shape"]
    phases = [ph for ph in phases if len(ph) >= 20 and "distribution" not in ph[0][0]]
    for i, ph in enumerate(phases):
        gaps = [(b[1] - a[2]) / 1e3 for a, b in zip(ph, ph[1:])]
        dur = [(r[2] - r[1]) / 1e3 for r in ph]
        label = names[i] if i < len(names) else f"phase {i}"
        print(f"{label:28s} kernels {len(ph):3d}  kernel median {statistics.median(dur):7.2f} us  "
              f"gap median {statistics.median(gaps):6.2f} us  (min {min(gaps):.2f}, max {max(gaps):.2f})")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run()


if __name__ == "__main__":
    main()

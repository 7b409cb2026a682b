"""Do back-to-back H2D copies on one stream run back-to-back? (run under rocprofv3)

    rocprofv3 --kernel-trace --memory-copy-trace -d out -o run -- \\
        python3 -m tools.studies.copy_pipe
    python -m tools.studies.copy_pipe --analyze out/run_results.db

The serving step is H2D-paced (8.6 MB of request arena per 16384-row step,
~157 us at ~54 GB/s), and the bench trace showed every copy starting 20-55 us
after the previous one ended. Phases (20 ms apart), 24 copies of 8.6 MB each:
  0  copies only
  1  copies + an event recorded after each
  2  1 + the compute stream waits each event and runs a ~100 us GEMM chain
  3  2 with the copy issued from a worker thread one step ahead of the waits
  4  2 with each copy split in two on two copy streams
  5  2 with the compute stream waiting on hipStreamWaitValue32 flags the copy
     stream writes (hipStreamWriteValue32) instead of events
  6+ the copies done by GPU waves reading the pinned host buffer
     (csrc/kernels/ingest.hip pull_host, launched on the copy stream):
     6 alone with 128 blocks, then like phase 2 with 32 / 128 / 512 blocks
 10  like phase 2 with consecutive copies alternating between two copy
     streams (one SDMA command's setup overlaps the other's transfer)
Printed per phase: median copy time, median idle time between copies, copy
throughput over the phase.
"""
from __future__ import annotations

import argparse
import ctypes
import statistics
import time

NBYTES = 8_621_120
N = 24


def run():
    import torch

    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32]
    hip.hipStreamWriteValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
    hosts = [torch.empty(NBYTES, dtype=torch.uint8).pin_memory() for _ in range(4)]
    devs = [torch.empty(NBYTES, dtype=torch.uint8, device=dev) for _ in range(4)]
    a = torch.randn(8192, 2752, device=dev, dtype=torch.bfloat16)
    w = torch.randn(2752, 1024, device=dev, dtype=torch.bfloat16)
    out = torch.empty(8192, 1024, device=dev, dtype=torch.bfloat16)
    flags = torch.zeros(N, dtype=torch.int32, device=dev)
    comp = torch.cuda.current_stream(dev)
    cp = torch.cuda.Stream(dev)
    cp2 = torch.cuda.Stream(dev)
    half = NBYTES // 2

    def work():
        torch.mm(a, w, out=out)
        torch.mm(a, w, out=out)

    def idle():
        torch.cuda.synchronize()
        time.sleep(0.02)

    work()
    idle()
    with torch.cuda.stream(cp):  # 0
        for i in range(N):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
    idle()
    with torch.cuda.stream(cp):  # 1
        for i in range(N):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
            torch.cuda.Event().record(cp)
    idle()
    for i in range(N):  # 2
        with torch.cuda.stream(cp):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cp)
        comp.wait_event(ev)
        work()
    idle()
    evs = []
    for i in range(N):  # 3: copies issued up front, then the waits
        with torch.cuda.stream(cp):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cp)
            evs.append(ev)
    for ev in evs:
        comp.wait_event(ev)
        work()
    idle()
    for i in range(N):  # 4
        e = []
        for st, lo in ((cp, 0), (cp2, half)):
            with torch.cuda.stream(st):
                devs[i % 4][lo:lo + half].copy_(hosts[i % 4][lo:lo + half], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
                e.append(ev)
        for ev in e:
            comp.wait_event(ev)
        work()
    idle()
    for i in range(N):  # 5
        with torch.cuda.stream(cp):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
        hip.hipStreamWriteValue32(ctypes.c_void_p(cp.cuda_stream), ctypes.c_void_p(flags[i:].data_ptr()), 1, 0)
        hip.hipStreamWaitValue32(ctypes.c_void_p(comp.cuda_stream), ctypes.c_void_p(flags[i:].data_ptr()), 1, 0,
                                 0xFFFFFFFF)  # hipStreamWaitValueGte
        work()
    idle()
    from distributed_tf_serving_amd import ops

    h = ops.hip()
    with torch.cuda.stream(cp):  # 6
        for i in range(N):
            h.pull_host(devs[i % 4], hosts[i % 4], NBYTES, 128)
    idle()
    for blocks in (32, 128, 512):  # 7, 8, 9
        for i in range(N):
            with torch.cuda.stream(cp):
                h.pull_host(devs[i % 4], hosts[i % 4], NBYTES, blocks)
                ev = torch.cuda.Event()
                ev.record(cp)
            comp.wait_event(ev)
            work()
        idle()
    ok = all(torch.equal(devs[i].cpu(), hosts[i]) for i in range(4))
    print("pull_host copies exact:", ok, flush=True)
    for i in range(N):  # 10
        st = cp if i % 2 == 0 else cp2
        with torch.cuda.stream(st):
            devs[i % 4].copy_(hosts[i % 4], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        comp.wait_event(ev)
        work()
    idle()


def analyze(db: str):
    import sqlite3

    c = sqlite3.connect(db)
    cps = [(s, e, z) for s, e, z in c.execute("select start, end, size from memory_copies order by start")
           if z >= NBYTES // 2 - 1024]
    cps += [(s, e, NBYTES) for n, s, e in c.execute("select name, start, end from kernels order by start")
            if "pull_host_kernel" in n]
    cps.sort()
    phases, cur = [], []
    for r in cps:
        if cur and r[0] - max(x[1] for x in cur) > 10_000_000:
            phases.append(cur)
            cur = []
        cur.append(r)
    if cur:
        phases.append(cur)
    kern = list(c.execute("select name, start, end from kernels order by start"))
    names = ["copies only", "copies + event", "copy/event/wait/compute", "copies issued up front",
             "split over two streams", "write/wait-value flags", "pull kernel alone (128)",
             "pull kernel + compute (32)", "pull kernel + compute (128)", "pull kernel + compute (512)",
             "alternating copy streams"]
    for i, ph in enumerate(phases):
        dur = [(e - s) / 1e3 for s, e, _ in ph]
        ends = sorted(e for _, e, _ in ph)
        starts = sorted(s for s, _, _ in ph)
        gaps = [(s2 - e1) / 1e3 for e1, s2 in zip(ends, starts[1:])] or [0.0]
        span = max(1.0, max(ends) - min(starts)) / 1e9
        gbps = sum(z for _, _, z in ph) / span / 1e9
        label = names[i] if i < len(names) else f"phase {i}"
        ks = [(n, s, e) for n, s, e in kern if min(starts) <= s <= max(ends) and "pull_host" not in n
              and n.startswith("Cijk")]
        kmed = statistics.median([(e - s) / 1e3 for _, s, e in ks]) if ks else 0.0
        print(f"{label:28s} copies {len(ph):3d}  copy median {statistics.median(dur):7.1f} us  "
              f"idle between {statistics.median(gaps):6.1f} us  phase {gbps:5.1f} GB/s  gemm median {kmed:6.1f} us")


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

"""Is the served step's 5.1 MB request copy bound by one SDMA engine or by the
PCIe link? Back-to-back pinned H2D copies of one step's bytes: one copy per
step on one stream, alternating over two streams (the StepRunner form), and
split in two halves issued at once on two streams (two engines in parallel).

    python -m tools.studies.h2d_split_study [--mb 5.1]
"""
from __future__ import annotations

import argparse
import json
import statistics

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=5.1)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    n = int(a.mb * (1 << 20)) // 256 * 256
    src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dst = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run(form):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        s2.wait_event(e0)
        for i in range(a.iters):
            d = dst[i % 4]
            if form == "one_stream":
                with torch.cuda.stream(s1):
                    d.copy_(src, non_blocking=True)
            elif form == "alternate":
                with torch.cuda.stream(s1 if i % 2 == 0 else s2):
                    d.copy_(src, non_blocking=True)
            else:
                h = n // 2
                with torch.cuda.stream(s1):
                    d[:h].copy_(src[:h], non_blocking=True)
                with torch.cuda.stream(s2):
                    d[h:].copy_(src[h:], non_blocking=True)
        s1.wait_stream(s2)
        e1.record(s1)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    forms = ["one_stream", "alternate", "split_halves"]
    t = {f: [] for f in forms}
    for _ in range(a.rounds):
        for f in forms:
            t[f].append(run(f))
    res = {"bytes": n}
    for f in forms:
        us = statistics.median(t[f])
        res[f + "_us"] = round(us, 2)
        res[f + "_GBps"] = round(n / us / 1e3, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

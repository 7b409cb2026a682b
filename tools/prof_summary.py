"""Summarise a rocprofv3 ``--kernel-trace --stats`` run (rocpd SQLite output)
into a markdown table for ``profiles/``.

    python -m tools.prof_summary gpurun_out/prof/run_results.db \
        --steps 110 --title "bench.py R=16" > profiles/bench_r16.md

Per kernel: calls, total / mean / min / max us, share of GPU busy time, and
per-step cost (total / steps). Also reports the steady-state step period
(median gap between consecutive launches of the step's last kernel) and the
idle gap between steps, the two numbers the serving pipeline is tuned on.
"""
from __future__ import annotations

import argparse
import re
import sqlite3
import statistics
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)  # drop argument lists
    name = name.replace("void ", "").replace("dtfs::kern::", "")
    return name[:90]


def summarize(db: str, steps: int = 0, title: str = "", last_kernel: str = "", from_kernel: str = "",
              step_kernel: str = "", min_us: float = 0.0) -> str:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end, duration from kernels order by start"))
    copies = list(c.execute("select name, start, end, duration, size from memory_copies order by start"))
    if from_kernel:  # drop start-up work (weight init, graph capture) before the first step kernel
        t0 = next((s for name, s, e, d in rows if from_kernel in name), None)
        if t0 is not None:
            rows = [r for r in rows if r[1] >= t0]
            copies = [r for r in copies if r[1] >= t0]
    agg = defaultdict(list)
    for name, s, e, d in rows:
        agg[_short(name)].append(d / 1e3)
    busy = sum(sum(v) for v in agg.values())
    out = [f"# {title or db}", ""]
    if rows:
        span = (rows[-1][2] - rows[0][1]) / 1e3
        out.append(f"kernels: {len(rows)} dispatches, GPU busy {busy:.0f} us over a {span:.0f} us trace span "
                   f"({100 * busy / max(span, 1e-9):.1f}% busy)")
    out += ["", "| kernel | calls | total us | mean us | min us | max us | % busy |" +
            (" us/step |" if steps else ""),
            "|---|---:|---:|---:|---:|---:|---:|" + ("---:|" if steps else "")]
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        t = sum(v)
        line = (f"| `{k}` | {len(v)} | {t:.0f} | {statistics.mean(v):.2f} | {min(v):.2f} | {max(v):.2f} | "
                f"{100 * t / max(busy, 1e-9):.1f} |")
        if steps:
            line += f" {t / steps:.2f} |"
        out.append(line)
    if copies:
        cagg = defaultdict(list)
        for name, s, e, d, size in copies:
            cagg[(name, size)].append(d / 1e3)
        out += ["", "| memory copy | bytes | calls | mean us | GB/s |", "|---|---:|---:|---:|---:|"]
        for (name, size), v in sorted(cagg.items(), key=lambda kv: -len(kv[1]))[:12]:
            m = statistics.mean(v)
            out.append(f"| {name} | {size} | {len(v)} | {m:.2f} | {size / max(m, 1e-9) / 1e3:.1f} |")
    if last_kernel:
        ends = [(s, e) for name, s, e, d in rows if last_kernel in name]
        if len(ends) > 4:
            period = statistics.median((b[1] - a[1]) / 1e3 for a, b in zip(ends, ends[1:]))
            out += ["", f"steady-state period between `{last_kernel}` launches: {period:.1f} us (median)"]
    if step_kernel:
        out += step_timeline(rows, copies, step_kernel, min_us)
    return "\n".join(out) + "\n"


def step_timeline(rows, copies, step_kernel: str, min_us: float) -> list:
    """Back-to-back steps: segment the kernel stream at every launch of
    ``step_kernel`` (the step's first kernel) and, for the pairs of consecutive
    segments whose ``step_kernel`` ran at least ``min_us`` (full-size steps),
    report the start-to-start period, the kernel time inside it and the idle
    rest - GPU-bound when idle ~ 0, host / copy-bound otherwise."""
    starts = [i for i, r in enumerate(rows) if step_kernel in r[0]]
    per, busy, idle, h2d, late, after = [], [], [], [], [], []
    big = [c for c in copies if c[4] >= (1 << 20) and "HOST_TO_DEVICE" in c[0]]  # the steps' request copies
    for a, b in zip(starts, starts[1:]):
        if rows[a][3] / 1e3 < min_us or rows[b][3] / 1e3 < min_us:
            continue
        t0, t1 = rows[a][1], rows[b][1]
        # union of kernel intervals in [t0, t1)
        ivs = sorted((max(s, t0), min(e, t1)) for _, s, e, _ in rows[a:b + 1] if s < t1)
        tot, cur_s, cur_e = 0, None, None
        for s, e in ivs:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        per.append((t1 - t0) / 1e3)
        busy.append(tot / 1e3)
        idle.append((t1 - t0 - tot) / 1e3)
        h2d.append(sum((min(e, t1) - max(s, t0)) for _, s, e, _, _ in copies if s < t1 and e > t0) / 1e3)
        # the request copy step b waited for: the last large H2D that landed
        # before b started; "late" = how long after the previous step's last
        # kernel ended it landed (> 0: the step waited for its bytes)
        fed = [c for c in big if c[2] <= t1]
        if fed and cur_e is not None:
            late.append((fed[-1][2] - cur_e) / 1e3)
            after.append((t1 - fed[-1][2]) / 1e3)
    if not per:
        return ["", f"no back-to-back full steps of `{step_kernel}` (>= {min_us} us)"]
    med = statistics.median
    return ["", f"back-to-back full steps ({len(per)} pairs, step starts at `{step_kernel}` >= {min_us} us): "
            f"period {med(per):.1f} us, kernels busy {med(busy):.1f} us, GPU idle {med(idle):.1f} us, "
            f"copy time inside the period {med(h2d):.1f} us (medians; p10/p90 period "
            f"{sorted(per)[len(per) // 10]:.1f} / {sorted(per)[9 * len(per) // 10]:.1f} us)"] + (
        [f"gap anatomy: the next step's request copy landed {med(late):.1f} us after the previous step's last kernel "
         f"ended (p10/p90 {sorted(late)[len(late) // 10]:.1f} / {sorted(late)[9 * len(late) // 10]:.1f}; > 0 = the "
         f"step waited for its H2D), and the step's first kernel started {med(after):.1f} us after that copy "
         f"landed (p10/p90 {sorted(after)[len(after) // 10]:.1f} / {sorted(after)[9 * len(after) // 10]:.1f})"]
        if late else [])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--title", default="")
    ap.add_argument("--last-kernel", default="", help="substring of the step's final kernel, for the step period")
    ap.add_argument("--from-kernel", default="", help="ignore everything before the first kernel matching this")
    ap.add_argument("--step-kernel", default="", help="substring of the step's FIRST kernel: step timeline")
    ap.add_argument("--min-us", type=float, default=0.0, help="full-size steps: --step-kernel at least this long")
    a = ap.parse_args()
    print(summarize(a.db, a.steps, a.title, a.last_kernel, a.from_kernel, a.step_kernel, a.min_us), end="")


if __name__ == "__main__":
    main()

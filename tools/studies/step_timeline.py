"""Per-step kernel timeline from a rocprofv3 kernel trace (rocpd SQLite):
for the steps anchored on ``--anchor`` (the step's big GEMM), each kernel's
start / end relative to the anchor's start, averaged over the last ``--last``
steps, plus the step period. Shows whether two lanes actually overlap
(step_program.py) and where the idle gaps are.

    python -m tools.studies.step_timeline gpurun_out/prof/run_results.db
"""
from __future__ import annotations

import argparse
import re
import sqlite3
import statistics
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name).replace("void ", "").replace("dtfs::kern::", "")
    return re.sub(r"^_ZN4dtfs4kern\d+", "", name)[:40]


def timeline(db: str, anchor: str = "gemm_8ph", last: int = 60, window_us: float = 400.0) -> str:
    c = sqlite3.connect(db)
    rows = [(_short(n), s / 1e3, e / 1e3) for n, s, e in c.execute("select name, start, end from kernels order by start")]
    try:  # SDMA copies too (H2D of the request arena): where they sit against the kernels
        rows += [("copy (H2D arena)" if size >= 1 << 20 else "copy (small)", s / 1e3, e / 1e3)
                 for s, e, size in c.execute("select start, end, size from memory_copies")]
        rows.sort(key=lambda r: r[1])
    except sqlite3.Error:
        pass
    anchors = [r for r in rows if anchor in r[0]]
    if len(anchors) < 3:
        return f"fewer than 3 '{anchor}' dispatches"
    anchors = anchors[-last - 1:-1]
    rel = defaultdict(list)
    for _, a0, _ in anchors:
        seen = defaultdict(int)
        for n, s, e in rows:
            if a0 - window_us / 2 <= s <= a0 + window_us:
                k = f"{n}#{seen[n]}" if seen[n] else n
                seen[n] += 1
                rel[k].append((s - a0, e - a0))
    periods = [b[1] - a[1] for a, b in zip(anchors, anchors[1:])]
    out = [f"anchor `{anchor}`: {len(anchors)} steps, period median {statistics.median(periods):.1f} us", "",
           "| kernel (relative to the anchor's start) | n | start us | end us | dur us |", "|---|---:|---:|---:|---:|"]
    for k, v in sorted(rel.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        if len(v) < len(anchors) // 2:
            continue
        s = statistics.median(x[0] for x in v)
        e = statistics.median(x[1] for x in v)
        d = statistics.median(x[1] - x[0] for x in v)
        out.append(f"| `{k}` | {len(v)} | {s:.1f} | {e:.1f} | {d:.1f} |")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--anchor", default="gemm_8ph")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    print(timeline(a.db, a.anchor, a.last))


if __name__ == "__main__":
    main()

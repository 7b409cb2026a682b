"""How far ahead of the GPU does the live server's launcher run? (rocprofv3
--kernel-trace --marker-trace with DTFS_TRACE=1, rocpd output)

    DTFS_TRACE=1 rocprofv3 --kernel-trace --marker-trace --memory-copy-trace -d out -o run \
        --output-format rocpd -- python3 bench.py --steps 100 --qps 0
    python -m tools.studies.launch_lead out/.../run_results.db --first resolve --big gemm_gather

For every full step (``--big`` kernel >= ``--min-us``) the step's first
kernel (``--first``) is matched with the ``live_launch`` marker range that
enqueued it (the last one that began before the kernel started). Printed
(medians over the steps): the lead = kernel start - launch range end (the
launcher finished enqueueing that long before the GPU started the step; ~0
or negative = the GPU waited for the host), the gap from the previous
step's last kernel end to this step's first kernel start, and where that
gap falls relative to the launch.
"""
from __future__ import annotations

import argparse
import bisect
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first", default="resolve")
    ap.add_argument("--big", default="gemm_gather")
    ap.add_argument("--min-us", type=float, default=80.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end from kernels order by start"))
    def ranges(msg):
        # roctx ranges: name = the API call, the message in extdata
        return sorted((s, e) for n, s, e, x in c.execute("select name, start, end, extdata from regions")
                      if n == msg or f'"message":"{msg}"' in (x or ""))

    regs, waits = ranges("live_launch"), ranges("live_wait")
    if not regs:
        raise SystemExit("no live_launch marker ranges (DTFS_TRACE=1 and --marker-trace?)")
    rs = [r[0] for r in regs]
    lead, gap, launch_after_prev_end = [], [], []
    prev_end = None
    for i, (n, s, e) in enumerate(ks):
        if a.first in n:
            # is this step a full one? (its big kernel follows)
            nxt = next((k for k in ks[i + 1:i + 4] if a.big in k[0]), None)
            if nxt and (nxt[2] - nxt[1]) / 1e3 >= a.min_us and prev_end is not None:
                j = bisect.bisect_right(rs, s) - 1
                if j >= 0:
                    ls, le = regs[j]
                    lead.append((s - le) / 1e3)
                    gap.append((s - prev_end) / 1e3)
                    launch_after_prev_end.append((le - prev_end) / 1e3)
        prev_end = max(prev_end or 0, e)
    med = statistics.median
    print(f"steps {len(lead)}: lead (first kernel start - launch end) median {med(lead):.1f} us "
          f"(p10 {sorted(lead)[len(lead) // 10]:.1f}, p90 {sorted(lead)[9 * len(lead) // 10]:.1f}); "
          f"gap to the previous kernel {med(gap):.1f} us; launch end - previous kernel end {med(launch_after_prev_end):.1f} us")
    if waits:
        d = [(e - s) / 1e3 for s, e in waits]
        print(f"live_wait ranges: {len(d)}, median {med(d):.1f} us")
    launches = [(e - s) / 1e3 for s, e in regs]
    print(f"live_launch ranges: {len(launches)}, median {med(launches):.1f} us")


if __name__ == "__main__":
    main()

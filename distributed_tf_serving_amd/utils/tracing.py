"""Tracing: roctx ranges from Python and the native runtime.

The reference's only instrumentation is wall-clock ``nanoTime`` around each
fan-out (reference DCNClient.java:141,198-199). Here:

* ``DTFS_TRACE=1`` turns on roctx ranges - from Python (:func:`trace_range`)
  and from the C++ serving loop (parse / launch / gpu_wait / encode per step,
  csrc/runtime/trace.cpp). Collect them together with the kernels:

      DTFS_TRACE=1 rocprofv3 --kernel-trace --marker-trace -d out -o run -- python3 bench.py

* :class:`StageTimer` accumulates per-stage wall time for the JSON summaries
  the benches and load generator print.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, Iterator

_ENABLED = os.environ.get("DTFS_TRACE", "0") == "1"


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    """roctx range (no-op unless DTFS_TRACE=1)."""
    if not _ENABLED:
        yield
        return
    from ..ops import native

    nat = native()
    nat.trace_push(name)
    try:
        yield
    finally:
        nat.trace_pop()


def mark(name: str) -> None:
    if _ENABLED:
        from ..ops import native

        native().trace_mark(name)


class StageTimer:
    """Accumulated wall time and counts per named stage."""

    def __init__(self):
        self.total: Dict[str, float] = defaultdict(float)
        self.count: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def stage(self, name: str) -> Iterator[None]:
        t0 = time.perf_counter()
        with trace_range(name):
            try:
                yield
            finally:
                self.total[name] += time.perf_counter() - t0
                self.count[name] += 1

    def summary_us(self) -> Dict[str, float]:
        return {k: round(v / max(1, self.count[k]) * 1e6, 2) for k, v in self.total.items()}

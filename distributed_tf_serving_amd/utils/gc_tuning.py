"""Keep CPython's cyclic garbage collector off the request path.

A serving process holds hundreds of thousands of long-lived objects (torch,
protobuf descriptors, the model registry); every generation-2 collection walks
all of them and stalls every Python thread for several milliseconds -- that is
what turns a sub-millisecond p50 into a tens-of-milliseconds p99 under open-loop
load (profiles/fixed_qps_grpc.md). The request path allocates few reference
cycles, so after start-up we move everything that exists into the permanent
generation (``gc.freeze``) and raise the generation-0 threshold so young
collections are rarer and only ever scan per-request garbage.

TF-Serving's counterpart is a C++ server with no tracing GC; this is the Python
front door's way of getting the same tail behaviour.
"""
from __future__ import annotations

import gc
import sys

_DEFAULT_GEN0 = 50_000
# CPython hands the GIL to a waiting thread only every switch interval (5 ms by
# default); a gRPC worker whose batch just completed can sit behind the
# load-generator or encoder thread for that long.
_DEFAULT_SWITCH_S = 5e-4


def freeze_heap(gen0_threshold: int = _DEFAULT_GEN0) -> dict:
    """Collect once, freeze the surviving heap, and raise the gen-0 threshold.

    Call after the model is loaded and warmed, before serving traffic. Returns
    a small report (frozen object count, thresholds) for logs and tests.
    """
    gc.collect()
    gc.freeze()
    _, g1, g2 = gc.get_threshold()
    gc.set_threshold(max(gen0_threshold, 1), g1, g2)
    return {"frozen": gc.get_freeze_count(), "threshold": gc.get_threshold()}


def tune_for_serving(gen0_threshold: int = _DEFAULT_GEN0, switch_interval_s: float = _DEFAULT_SWITCH_S) -> dict:
    """:func:`freeze_heap` plus a shorter GIL switch interval (serving processes)."""
    rep = freeze_heap(gen0_threshold)
    if switch_interval_s > 0:
        sys.setswitchinterval(switch_interval_s)
    rep["switch_interval_s"] = sys.getswitchinterval()
    return rep


def unfreeze_heap() -> None:
    """Undo :func:`freeze_heap` (tests; a server that reloads models in place)."""
    gc.unfreeze()
    gc.set_threshold(700, 10, 10)

"""NUMA placement helpers (csrc/runtime/numa.cpp, utils/affinity.py) on the
CPU box: node discovery from sysfs, binding every thread of the process (and
threads created later) to a CPU set, node-bound allocations (page placement
read back with move_pages), and the no-op paths (CPU device, unknown PCI id).
The GPU path (the GPU's bus id -> node, hipHostRegister of node-local arenas)
runs in tests/test_live_gpu.py."""
import os
import threading

import pytest
import torch

from distributed_tf_serving_amd.ops import native
from distributed_tf_serving_amd.utils import affinity


def _thread_cpus(tid):
    with open(f"/proc/self/task/{tid}/status") as f:
        line = next(ln for ln in f if ln.startswith("Cpus_allowed_list"))
    out = set()
    for part in line.split(":")[1].strip().split(","):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def test_node_discovery_and_unknown_pci():
    n = native()
    assert n.numa_node_count() >= 1
    cpus0 = n.numa_node_cpus(0)
    if os.path.exists("/sys/devices/system/node/node0"):
        assert cpus0 and all(c >= 0 for c in cpus0)
    assert n.numa_node_cpus(-1) == []
    assert n.pci_numa_node("0000:ff:1f.7") == -1


def test_bind_every_thread_and_inherit():
    n = native()
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 2:
        pytest.skip("needs two CPUs")
    target = allowed[:1]
    ev = threading.Event()
    t_old = threading.Thread(target=ev.wait)  # exists before the bind
    t_old.start()
    try:
        bound = n.bind_process_cpus(target)
        assert bound >= 2
        tids = os.listdir("/proc/self/task")
        assert all(_thread_cpus(t) == set(target) for t in tids)
        seen = {}
        t_new = threading.Thread(target=lambda: seen.update(cpus=os.sched_getaffinity(0)))  # inherits
        t_new.start()
        t_new.join()
        assert seen["cpus"] == set(target)
    finally:
        n.bind_process_cpus(allowed)
        ev.set()
        t_old.join()
    assert os.sched_getaffinity(0) == set(allowed)


def test_node_bound_allocation():
    n = native()
    t = n.alloc_on_node(3 << 20, 0)
    assert t.dtype == torch.uint8 and t.numel() == 3 << 20 and int(t[12345]) == 0
    t[:] = 7
    node = n.page_numa_node(t, 0)
    if node == -1:
        pytest.skip("move_pages not permitted here")
    assert node == 0 and n.page_numa_node(t, (3 << 20) - 1) == 0
    del t


def test_place_rank_noop_on_cpu_and_place_on_node():
    assert affinity.place_rank(torch.device("cpu")) == {"node": -1}
    allowed = os.sched_getaffinity(0)
    try:
        info = affinity.place_on_node(0)
        if info.get("note"):
            pytest.skip(info["note"])
        assert info["threads_bound"] >= 1 and affinity.current_node() == 0
        assert os.sched_getaffinity(0) <= set(native().numa_node_cpus(0))
    finally:
        native().bind_process_cpus(sorted(allowed))
        affinity._placement.clear()
        affinity._placement["node"] = -1

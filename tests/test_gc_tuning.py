"""utils/gc_tuning.py: the serving processes freeze their start-up heap so
generation-2 collections never walk it on the request path."""
import gc

import sys

from distributed_tf_serving_amd.utils.gc_tuning import freeze_heap, tune_for_serving, unfreeze_heap


def test_freeze_and_unfreeze():
    before = gc.get_threshold()
    try:
        rep = freeze_heap(gen0_threshold=12345)
        assert rep["frozen"] > 0 and gc.get_freeze_count() == rep["frozen"]
        assert gc.get_threshold()[0] == 12345
        # objects created after the freeze are still collected
        a = []
        a.append(a)
        del a
        assert gc.collect() >= 1
    finally:
        unfreeze_heap()
        gc.set_threshold(*before)
    assert gc.get_freeze_count() == 0


def test_entry_points_opt_out_flag():
    from distributed_tf_serving_amd.client import loadgen
    from distributed_tf_serving_amd.serving import server
    for mod in (loadgen, server):
        assert "--no-gc-freeze" in open(mod.__file__).read()


def test_tune_for_serving_sets_switch_interval():
    before, sw = gc.get_threshold(), sys.getswitchinterval()
    try:
        rep = tune_for_serving(switch_interval_s=1e-3)
        assert abs(rep["switch_interval_s"] - 1e-3) < 1e-9
    finally:
        unfreeze_heap()
        gc.set_threshold(*before)
        sys.setswitchinterval(sw)

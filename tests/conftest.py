import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built _hip extension")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    # the host runtime (_native) is needed by CPU tests too; build it in-tree once
    from distributed_tf_serving_amd.ops import _loader

    _loader.native()
    yield


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_tf_serving_amd.ops import _loader

    _loader.hip()  # fail loudly if the kernels are not built
    return torch.device("cuda:0")

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the in-tree HIP kernel library")
    config.addinivalue_line("markers", "slow: multi-process or long-running CPU test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        if torch.cuda.is_available():
            return
    except ImportError:  # the CI lint job runs the torch-free manifest tests only
        pass
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def kernels():
    """Build (if needed) and load the gfx950 kernel library; fail loudly if it is missing."""
    from nanosandbox_amd.build import build_all
    from nanosandbox_amd.ops import _lib

    build_all(verbose=False)
    return _lib.lib()

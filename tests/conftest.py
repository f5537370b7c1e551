import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: larger CPU sizes")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("ZKM_FORCE_GPU_TESTS"):
        return
    try:
        import torch  # noqa: F401  (device discovery only)
        have = torch.cuda.is_available()
    except Exception:
        have = False
    if not have:
        skip = pytest.mark.skip(reason="no GPU visible")
        for it in items:
            if "gpu" in it.keywords:
                it.add_marker(skip)

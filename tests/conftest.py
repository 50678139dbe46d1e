import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu() -> bool:
    # device_count() does not initialise HIP on this image (is_available() does):
    # GPU tests that spawn rank processes must run before the parent touches
    # the device (tests/test_00_tp_gpu.py)
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU available")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

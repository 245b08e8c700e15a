import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# keep the service quiet and CPU-friendly in tests
os.environ.setdefault("LOG_LEVEL", "WARNING")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)

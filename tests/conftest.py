import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
DATA = os.path.join(GOLDEN, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def has_gpu_device():
    # Decided from the device node only: on a GPU box the gpu tests always run, so a
    # missing/broken HIP extension fails them loudly instead of skipping.
    return os.path.exists("/dev/kfd")


def pytest_collection_modifyitems(config, items):
    if has_gpu_device():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# multi-process operator tests (minutes, many replicas): run after every
# kernel / graph / collective numerics test, so one stalled job can never
# hide the numerics results behind `-x`
_LAST = ("test_e2e_gpu.py", "test_e2e_cpu.py", "test_restart_wave.py")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: multi-process / long-running test")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: 1 if os.path.basename(str(it.fspath)) in _LAST else 0)  # stable
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

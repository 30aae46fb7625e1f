import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")
    # Multi-process tests fork their ranks from a forkserver that must start before
    # this process initialises a GPU (a GPU-initialised process must never exec).
    from dist_gpu_accelerated_tree_search_amd.parallel.launch import warm_forkserver

    warm_forkserver()


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)

import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    # under pytest-xdist every worker would otherwise start a full intra-op thread pool
    n = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
    if n:
        import torch
        torch.set_num_threads(max(1, (os.cpu_count() or 8) // int(n)))
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _cloud():
    import h2o3_amd
    h2o3_amd.init(verbose=False)
    yield

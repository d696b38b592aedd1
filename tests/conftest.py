import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _cloud():
    import h2o3_amd
    h2o3_amd.init(verbose=False)
    yield

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "another-cuda-sift_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsift_hip.so on the GPU)")
    config.addinivalue_line("markers", "slow: multi-second CPU oracle runs")


@pytest.fixture(scope="session")
def sift():
    import sift_amd

    return sift_amd


@pytest.fixture(scope="session")
def oracle():
    import oracle_binding

    return oracle_binding

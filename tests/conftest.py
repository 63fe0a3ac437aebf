import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# before any test module imports torch: the package sets HIP's graph-capture mode ahead of HIP's
# initialisation (zbot_lab_amd/__init__.py), so the runner's HIP graphs are on whatever the order
# in which pytest collects the test files
import zbot_lab_amd  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs through libzbot.so")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def robot():
    from zbot_lab_amd import model as zm
    return zm.load_model()


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm GPU is visible")
    from zbot_lab_amd import build
    build.build()
    return torch.device("cuda:0")

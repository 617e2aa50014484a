import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libmonkeypose.so")
    config.addinivalue_line("markers", "slow: long-running CPU oracle test")


def load_pkg():
    """The product package lives in a hyphenated directory: import it by name via importlib."""
    return importlib.import_module("monkey-pose_amd")


@pytest.fixture(scope="session")
def mp():
    return load_pkg()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")

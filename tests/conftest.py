import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libsem_hip.so")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def gll():
    return load_golden("gll.npz")


@pytest.fixture(scope="session")
def poisson_action():
    return load_golden("poisson_action.npz")


@pytest.fixture(scope="session")
def poisson_solution():
    return load_golden("poisson_solution.npz")


@pytest.fixture(scope="session")
def axisym_action():
    return load_golden("axisym_action.npz")


@pytest.fixture(scope="session")
def tensor_ops():
    return load_golden("tensor_ops.npz")


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb else 1.0)


@pytest.fixture(scope="session")
def axisym_ns():
    return load_golden("axisym_ns.npz")


@pytest.fixture(scope="session")
def hex_golden():
    return load_golden("hex.npz")

"""Shared test setup. `-m gpu` tests need a real MI355X (they call through the
C-ABI into the HIP kernels); everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "point-cloud-signed-distance_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs the HIP kernels through the C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def irb():
    from flash import Models
    return Models.irb140()


@pytest.fixture(scope="session")
def m64():
    from flash import Models
    return Models.arm_grid()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.load()
    return oracle


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))

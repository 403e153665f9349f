import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhbmi.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def golden(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle  # test infrastructure (checker) only

    return Oracle()


@pytest.fixture(scope="session")
def hbmi():
    """The product library; GPU tests fail (not skip) without a device."""
    from hb_mcmc_amd import _lib

    lib = _lib.lib()
    if not _lib.device_available():
        pytest.fail("no HIP device visible: GPU parity tests need an MI355X")
    return lib

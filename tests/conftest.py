import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpsn_lk.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # tests are allowed to use the oracle as the checker

    oracle.lib()
    return oracle

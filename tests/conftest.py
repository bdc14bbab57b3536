import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# The product library is loaded before any test module imports torch: it binds
# the ROCm runtime it was built against (/opt/rocm) and gives it the names
# torch's libraries ask for, so every test process maps ONE HIP/HSA/RCCL
# runtime whatever the module order (psn_lk_runtime_info, include/psn_lk.h).
if os.path.exists(os.path.join(ROOT, "mcmtt_opticalflow_amd", "lib", "libpsn_lk.so")):
    from mcmtt_opticalflow_amd import _lib as _product_lib

    _product_lib.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpsn_lk.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # tests are allowed to use the oracle as the checker

    oracle.lib()
    return oracle

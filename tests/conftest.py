import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "hkd-mpc_amd"), os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP product path)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built_artifacts():
    """Make sure the oracle (test infrastructure) is compiled before any test uses it."""
    import oracle_lib
    if not os.path.exists(oracle_lib.LIB_PATH):
        oracle_lib.build()
    yield


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "hkd_model_golden.npz")))

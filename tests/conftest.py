import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C-ABI on cuda:0)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def text_fixture():
    return dict(np.load(os.path.join(GOLDEN, "text_svo.npz")))


@pytest.fixture(scope="session")
def text_svo(text_fixture):
    from raytracingtest_amd.svo_data import SVOData
    z = text_fixture
    return SVOData.from_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"], z["normal_code"])


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.lib()
    return oracle

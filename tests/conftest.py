import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")
    config.addinivalue_line("markers", "slow: large instance")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def native():
    from alllsatisfiabilitysolver_amd import _native

    _native.build()
    return _native

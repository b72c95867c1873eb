import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")

# The library, and with it the ROCm runtime it is built against, is loaded before any test
# module imports torch (whose wheel bundles another HIP runtime under the same soname; the
# first one loaded serves the process: INTEGRATION.md §3).
try:
    from alllsatisfiabilitysolver_amd import _native as _alll_native

    _alll_native.lib()
except Exception:  # not built yet: the ABI tests report it
    pass


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

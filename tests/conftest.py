import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device 0); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the native libraries once per session (incremental, no GPU needed;
    CCSX_NO_BUILD=1: use the libraries as they are, e.g. a variant under test)."""
    if os.environ.get("CCSX_NO_BUILD"):
        yield
        return
    from ccsx_amd.build import build_oracle, build_product
    build_product()
    build_oracle()
    yield


@pytest.fixture(scope="session")
def engine():
    import ccsx_amd as cx
    e = cx.Engine(0)
    yield e
    e.close()

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_c
    oracle_c.build()
    return oracle_c


@pytest.fixture(scope="session")
def nkv():
    """The HIP library + one context on device 0 (GPU tests only)."""
    from nakevaleng_amd import build as b
    b.build()
    from nakevaleng_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: GPU tests must run on an MI355X")
    ctx = _lib.Context(0)
    yield _lib, ctx
    ctx.close()


def pytest_terminal_summary(terminalreporter):
    """Say which library the run used and whether it was built from these sources."""
    try:
        from nakevaleng_amd import build as b
    except Exception:  # pragma: no cover
        return
    if b.last_status:
        terminalreporter.write_line("nakevaleng_amd: " + b.last_status)

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import Oracle
    return Oracle.get()


@pytest.fixture
def knob(monkeypatch):
    """Set one NAD_* switch for this test: the library reads them once (never per call), so re-read after setting."""
    from neural_amd import _lib

    def set_(name, value):
        if value is None:
            monkeypatch.delenv(name, raising=False)
        else:
            monkeypatch.setenv(name, str(value))
        _lib.reload_knobs()
    return set_


@pytest.fixture(autouse=True)
def _knobs_follow_environment():
    """Autouse fixtures tear down last: by then monkeypatch has restored the environment, so the library's switches go
    back to it too."""
    yield
    from neural_amd import _lib
    if _lib._LIB is not None:
        _lib.reload_knobs()

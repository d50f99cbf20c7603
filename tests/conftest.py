import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def _has_gpu() -> bool:
    try:
        from flipcomplexityempirical_amd import _lib
        return _lib.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not _has_gpu():
        pytest.fail("GPU test selected but no HIP device / libflipchain.so is available")
    return True


@pytest.fixture(scope="session")
def cref():
    from oracle import flipref
    flipref.build_lib()
    return flipref.CRef()


@pytest.fixture(scope="session")
def sec11():
    from flipcomplexityempirical_amd import graphs
    return graphs.sec11_graph()


@pytest.fixture(scope="session")
def frank():
    from flipcomplexityempirical_amd import graphs
    return graphs.frank_graph()

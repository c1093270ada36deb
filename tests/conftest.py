"""pytest configuration: the `gpu` marker, the package alias and the oracle (checker)."""
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import __graft_entry__  # noqa: E402

pkg = __graft_entry__.load_package()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libtog.so")


@pytest.fixture(scope="session")
def tog():
    return pkg


@pytest.fixture(scope="session")
def oracle():
    return __graft_entry__.load_oracle()


def gpu_available():
    try:
        lib = pkg.abi.load_library()
        return lib.tog_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Fails loudly (no silent CPU fallback) when the HIP library or device is missing."""
    lib = pkg.abi.load_library()
    assert lib.tog_device_count() > 0, "no HIP device visible"
    return lib

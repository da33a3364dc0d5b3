import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "algo-dsp_amd"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU; runs through the HIP C ABI")


@pytest.fixture(scope="session")
def gpu():
    """Session guard for GPU tests: the HIP library must load and see a device."""
    from algodsp import _lib

    n = _lib.device_count()
    if n < 1:
        pytest.fail("GPU test collected but no HIP device is visible")
    return n

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) -- run with -m gpu")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    oracle_lib.build()
    return oracle_lib


@pytest.fixture(scope="session", params=["masks", "swar"])
def emu(request):
    """The device per-line code on the CPU, once with the byte-class masks of
    the kernel's LDS path and once with the SWAR scanners of its HBM path."""
    import emu_lib
    emu_lib.build()
    emu_lib.lib().emu_set_masks(1 if request.param == "masks" else 0)
    return emu_lib


@pytest.fixture(scope="session")
def vectors():
    import golden_check
    return golden_check.load_vectors()


@pytest.fixture(scope="session")
def demolog_lines():
    path = os.path.join(ROOT, "tests", "golden", "hackers-access.log")
    with open(path, "rb") as f:
        data = f.read()
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return lines

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


@pytest.fixture(scope="session")
def emu():
    import emu_lib
    emu_lib.build()
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

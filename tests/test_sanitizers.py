"""The oracle and the test-only emulation of the device code (lp_device.h +
plan.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer: a subset of the
CPU parity tests through tools/asan_check.sh (host code only; there are no GPU
sanitizers on this pool).  The full selection: tools/asan_check.sh with no
arguments (about 2 minutes)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_parity_under_asan_ubsan():
    if not shutil.which("gcc") or not os.path.exists(subprocess.run(
            ["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()):
        pytest.skip("no libasan")
    r = subprocess.run([os.path.join(ROOT, "tools", "asan_check.sh"),
                        "golden or synthetic_config2 or utf8 or upstream or setup or resilient or cookies"],
                       capture_output=True, text=True, timeout=850)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "passed" in r.stdout and "failed" not in r.stdout, tail

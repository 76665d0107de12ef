"""Host sanitizers: the C oracle and the C-ABI library's host
side built with AddressSanitizer + UndefinedBehaviorSanitizer (`make asan`;
device code is compiled normally, sanitizers apply to host code only) and
driven without a GPU: the oracle's MH and MALA sweeps on clipped windows and
edge-of-box proposals (scripts/asan/oracle_driver.c), and every C entry
point's argument validation (scripts/asan/capi_driver.cpp).  A sanitizer
report fails the test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("gcc / hipcc not available")
    jobs = max(1, min(int(os.environ.get("MAX_JOBS", "8")), 8))
    r = subprocess.run(["make", "-C", ROOT, f"-j{jobs}", "asan"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return ASAN


def _run(path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    r = subprocess.run([path], capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


@pytest.mark.timeout(1200)
def test_oracle_under_asan_ubsan(built):
    assert "ok" in _run(os.path.join(built, "oracle_driver"))


@pytest.mark.timeout(1200)
def test_capi_validation_under_asan_ubsan(built):
    assert "0 failure(s)" in _run(os.path.join(built, "capi_driver"))

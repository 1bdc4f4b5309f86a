"""Sanitizer runs of the host code ("race detection /
sanitizers"): `make asan` builds the CPU oracle (oracle/_build_asan) and the
C++ drop-in surface's host code (detector_cxx.cpp, multi_cxx.cpp, linked into
the CPU orchestration test tests/cpp/test_multi.cpp) with
-fsanitize=address,undefined.  HIP kernels are not instrumented (GPU ASan is
not available on the GPU pool)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_ENV = {"ASAN_OPTIONS": "abort_on_error=0:halt_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"}

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")


@pytest.fixture(scope="module")
def asan_build():
    r = subprocess.run(["make", "-C", ROOT, "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lib = os.path.join(ROOT, "oracle", "_build_asan", "libsift_oracle.so")
    syms = subprocess.run(["nm", "-D", lib], capture_output=True, text=True, check=True).stdout
    assert "__asan_" in syms and "__ubsan_" in syms, "oracle/_build_asan is not a sanitizer build"
    return lib


def test_multi_orchestration_under_asan(asan_build):
    """The C++ MultiDetector / crossMatch orchestration with injected fakes,
    host code instrumented (leak checking on)."""
    exe = os.path.join(ROOT, "another-cuda-sift_amd", "lib", "asan", "test_multi")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=dict(os.environ, **ASAN_ENV))
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "multi orchestration ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_oracle_suite_under_asan(asan_build):
    """tests/test_oracle.py (golden fixtures, invariants, knn-2) against the
    sanitizer build of the oracle, in a Python process with libasan preloaded
    (Python's own allocations are not leak-checked)."""
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True,
                             check=True).stdout.strip()
    env = dict(os.environ, SIFT_ORACLE_BUILD="_build_asan", LD_PRELOAD=libasan,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS=ASAN_ENV["UBSAN_OPTIONS"])
    r = subprocess.run([sys.executable, "-m", "pytest", os.path.join(ROOT, "tests", "test_oracle.py"), "-x", "-q",
                        "-p", "no:cacheprovider"], capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed" in r.stdout and "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr

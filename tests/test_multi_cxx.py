"""The C++ multi-GPU surface (include/sift_cuda/MultiDetector.hh): its
orchestration on CPU with injected fakes (tests/cpp/test_multi.cpp, linked
against libsift_cuda.so), and the exported C ABI entry points it uses."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "another-cuda-sift_amd", "lib")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_multi_orchestration_with_fakes(tmp_path):
    exe = tmp_path / "test_multi"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-pthread", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_multi.cpp"), "-o", str(exe), "-L", LIB, "-lsift_cuda",
                    "-lsift_hip", f"-Wl,-rpath,{LIB}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "multi orchestration ok" in r.stdout


def test_multi_symbols_exported():
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(LIB, "libsift_cuda.so")], capture_output=True,
                         text=True, check=True).stdout
    for s in ["sift_cuda::MultiDetector::detectAll(", "sift_cuda::crossMatch(", "sift_cuda::rcclAllGather(",
              "sift_cuda::copyAllGather(", "sift_cuda::hipBatchMatch(", "sift_cuda::Detector::Detector(CudaSiftConfig const&, int)"]:
        assert s in out, s

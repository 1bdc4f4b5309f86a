"""OpenCV interop row on CPU: the numpy field mapping of
sift_amd.cv (Conversion.cc:21-58 semantics), and the C++ header
include/cvUtils/Conversion.hh: refused with a clear error where OpenCV is
absent (this image), compiled where it is present."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from sift_amd import cv as scv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_keypoint_fields_mapping():
    k = np.array([[1.5, 2.25, 1.0], [10.0, 20.0, 2.0], [3.0, 4.0, 1.0]], np.float32)
    octave = (1 << 8) | (2 << 16) | 0xff  # layer 1, octave -1 packed as OpenCV does
    f = np.array([[octave, 3.5, 0.02, 90.0], [2 << 8, 7.0, 0.05, 0.0], [0, 1.0, 0.1, 359.5]], np.float32)
    out = scv.keypoint_fields(k, f)
    assert np.array_equal(out["x"], k[:, 0]) and np.array_equal(out["y"], k[:, 1])
    assert out["octave"][0] == octave and out["octave"].dtype == np.int32
    assert np.array_equal(out["size"], f[:, 1]) and np.array_equal(out["response"], f[:, 2])
    assert np.array_equal(out["angle"], f[:, 3])
    assert len(scv.keypoint_fields(k, f, size=2)["x"]) == 2
    with pytest.raises(ValueError):
        scv.keypoint_fields(k, f[:2])


def test_descriptor_matrix_and_dmatch():
    d = (np.arange(3 * 128) % 256).astype(np.float16)
    m = scv.descriptor_matrix(d, 2)
    assert m.shape == (2, 128) and m.dtype == np.float32 and m[1, 0] == 128.0
    assert scv.descriptor_matrix(d, 10).shape == (3, 128)
    assert scv.dmatch_triples([3, -1, 0, -1]) == [(0, 3, 0.0), (2, 0, 0.0)]


def test_cv2_builders_match_fields():
    cv2 = pytest.importorskip("cv2")
    k = np.array([[1.5, 2.25, 1.0]], np.float32)
    f = np.array([[256, 3.5, 0.02, 90.0]], np.float32)
    kp = scv.to_cv_keypoints(k, f)[0]
    assert (kp.pt, kp.size, kp.angle, kp.octave) == ((1.5, 2.25), 3.5, 90.0, 256)
    assert scv.to_cv_dmatches([2, -1])[0].trainIdx == 2


def test_cvutils_header_gated(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    src = tmp_path / "t.cpp"
    src.write_text('#include "cvUtils/Conversion.hh"\nint main() { return (int)OpencvUtils::cvtMatchToDMatch({1, -1}).size() - 1; }\n')
    r = subprocess.run([cxx, "-std=c++17", "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o", str(tmp_path / "t.o")],
                       capture_output=True, text=True)
    has_cv = subprocess.run([cxx, "-std=c++17", "-x", "c++", "-E", "-"], input="#include <opencv2/core.hpp>\n",
                            capture_output=True, text=True).returncode == 0
    if has_cv:
        assert r.returncode == 0, r.stderr
    else:
        assert r.returncode != 0 and "needs OpenCV" in r.stderr

"""C-ABI boundary checks without a GPU.

* libsift_hip.so loads and exports every function include/sift_hip.h declares;
  libsift_cuda.so exports the sift_cuda:: drop-in surface
  (include/sift_cuda/*.hh, reference Detector.hh / Match.cuh).
* The public headers compile with a plain C / C++ compiler (no HIP headers).
* Host-side logic that runs before any device call: default config (the
  reference's CudaSiftConfig.hh defaults), octave geometry against the oracle,
  argument validation and the loud failure when no GPU is present.
"""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "another-cuda-sift_amd", "lib")


def header_functions():
    text = open(os.path.join(INC, "sift_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\**\s+\**\s*(sift_\w+)\s*\(", text, flags=re.M)))


def exported(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_declares_expected_surface():
    fns = header_functions()
    for f in ["sift_hip_create", "sift_hip_destroy", "sift_hip_warmup", "sift_hip_detect", "sift_hip_copy_to_host",
              "sift_hip_results_device", "sift_hip_match_device", "sift_hip_match_host", "sift_hip_last_error",
              "sift_hip_detect_u8", "sift_hip_submit", "sift_hip_wait", "sift_hip_detect_device_fmt"]:
        assert f in fns
    assert len(fns) >= 30


def test_libsift_hip_exports_every_declared_symbol(sift):
    lib = os.path.join(LIBDIR, "libsift_hip.so")
    assert os.path.exists(lib)
    syms = exported(lib)
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing
    L = sift.lib()  # loads through ctypes as the Python surface does
    for f in header_functions():
        assert hasattr(L, f)


def test_libsift_cuda_exports_dropin_surface():
    lib = os.path.join(LIBDIR, "libsift_cuda.so")
    out = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    for s in ["sift_cuda::Detector::Detector(CudaSiftConfig const&)",
              "sift_cuda::Detector::gpuWarmUpAndAllocate()",
              "sift_cuda::Detector::detectAndCompute(Image<float> const&)",
              "sift_cuda::Detector::copyToHost(bool)",
              "sift_cuda::Detector::setExactDescriptors(bool)",
              "sift_cuda::matchBruteForce("]:
        assert s in out, s


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_headers_compile_without_hip(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "sift_hip.h"\nint main(void){sift_hip_config c; (void)c; return 0;}\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-I", INC, str(c)], check=True)
    cc = tmp_path / "t.cc"
    cc.write_text("".join(f'#include "sift_cuda/{h}"\n' for h in sorted(os.listdir(os.path.join(INC, "sift_cuda"))))
                  + "int main(){ CudaSiftConfig c; (void)c; return 0; }\n")
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", "-I", INC, str(cc)], check=True)


def test_version_and_default_config(sift):
    v = sift.version()
    assert "abi=1" in v and "gfx950" in v
    assert "build=default" in v and sift.is_default_build(), v  # no A/B macros in the shipped library
    cfg = sift.CudaSiftConfig(col_width=640, row_width=480)
    # Reference defaults (CudaSiftConfig.hh:3-14).
    assert (cfg.numFeatures, cfg.numOctaveLayers, cfg.contrastThreshould, cfg.edgeThreshould, cfg.sigma) == \
        (5000, 3, 0.04, 10.0, 1.6)
    c = sift._Config()
    sift.lib().sift_hip_default_config(ctypes.byref(c), 640, 480)
    assert (c.col_width, c.row_width, c.numOctaveLayers, c.numOctaves) == (640, 480, 3, 0)
    assert abs(c.sigma - 1.6) < 1e-12 and abs(c.contrastThreshould - 0.04) < 1e-12


@pytest.mark.parametrize("w,h,upscale,nOct", [(1920, 1200, False, 0), (1920, 1200, False, 3), (752, 480, True, 0),
                                              (257, 191, True, 0), (1600, 900, False, 0)])
def test_octave_geometry_matches_oracle(sift, oracle, w, h, upscale, nOct):
    """Geometry is host logic computed at create time (no device call)."""
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, upscale=upscale, numOctaves=nOct)
    det = sift.Detector(cfg, device=0)
    p = oracle.from_config(cfg)
    assert det.nOctaves == oracle.num_octaves(w, h, p)
    for o in range(det.nOctaves):
        ow, oh, pitch = det.octave_dims(o)
        assert (ow, oh) == oracle.octave_dims(w, h, p, o)
        assert pitch >= ow and pitch % 64 == 0  # rows start on 256-byte boundaries


def test_invalid_arguments_fail_with_status(sift):
    L = sift.lib()
    h = ctypes.c_void_p()
    c = sift._Config()
    L.sift_hip_default_config(ctypes.byref(c), 0, 480)
    assert L.sift_hip_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1  # SIFT_HIP_ERR_INVALID
    assert L.sift_hip_last_error()
    L.sift_hip_default_config(ctypes.byref(c), 64, 64)
    c.numOctaveLayers = 0
    assert L.sift_hip_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1
    assert L.sift_hip_create(None, 0, ctypes.byref(h)) == -1
    assert L.sift_hip_destroy(None) == 0  # like free(NULL): a no-op
    k3 = ctypes.c_void_p()
    assert L.sift_hip_results_host(None, ctypes.byref(k3), None, None, None) != 0  # null handle: a status, no crash


def test_no_gpu_fails_loudly(sift):
    """Without a device the product path raises; there is no CPU fallback."""
    n = ctypes.c_int(-1)
    rc = sift.lib().sift_hip_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    det = sift.Detector(sift.CudaSiftConfig(col_width=64, row_width=64))
    with pytest.raises(sift.SiftHipError):
        det.gpuWarmUpAndAllocate()
    with pytest.raises(sift.SiftHipError):
        det.detectAndCompute(np.zeros((64, 64), np.float32))


def test_python_surface_mirrors_reference(sift):
    for name in ["gpuWarmUpAndAllocate", "detectAndCompute", "copyToHost"]:
        assert callable(getattr(sift.Detector, name))
    assert callable(sift.matchBruteForce)
    for f in ["col_width", "row_width", "numFeatures", "numOctaveLayers", "contrastThreshould", "edgeThreshould",
              "sigma", "upscale"]:
        assert hasattr(sift.CudaSiftConfig(col_width=8, row_width=8), f)


def test_batch_host_logic(sift):
    """sift_hip_set_batch limits and call order (no GPU work involved)."""
    L = sift.lib()
    h = ctypes.c_void_p()
    c = sift._Config()
    L.sift_hip_default_config(ctypes.byref(c), 64, 64)
    assert L.sift_hip_create(ctypes.byref(c), 0, ctypes.byref(h)) == 0
    try:
        assert L.sift_hip_set_batch(h, 0) == -1
        assert L.sift_hip_set_batch(h, 65) == -1
        assert L.sift_hip_set_batch(h, 4) == 0
        n = ctypes.c_int()
        assert L.sift_hip_batch_capacity(h, ctypes.byref(n)) == 0 and n.value == 4
        # before sift_hip_warmup: out of order, refused before any device call
        assert L.sift_hip_detect_batch_device(h, ctypes.c_void_p(16), 2, 0, 0, 0, None) == -3
        assert L.sift_hip_batch_results_device(h, 0, None, None, None, None, None) == -3
    finally:
        L.sift_hip_destroy(h)
    assert L.sift_hip_set_batch(None, 2) == -1


def test_match_plan_host_only(sift):
    """sift_hip_match_plan needs no GPU: single pairs use 4-wave workgroups and
    >= 4-tile splits; C5 (56 pairs of 2000 x 2000) runs one split per query
    block; the ragged batched case of test_gpu_parity has S > 1."""
    S, nw = sift.Matcher.plan(2000, 2000, 1)
    assert nw == 4 and 1 < S <= 16
    assert sift.Matcher.plan(2000, 2000, 56) == (1, 8)
    assert sift.Matcher.plan(2000, 2500, 8)[0] > 1
    with pytest.raises(sift.SiftHipError):
        sift.Matcher.plan(10, 10, 0)


def test_capacities_sized_to_the_frame(sift):
    """Per-frame capacities follow the geometry and numFeatures (host-only,
    before warm-up): the reference-config 752x480 handle's result ring is
    numFeatures + 25 %, its candidate list 1/8 of the scale-space samples;
    maxKeypoints overrides the result capacity; numFeatures = 0 sizes results
    from the pyramid's pixels.  Every capacity stays within the old fixed caps."""
    d = sift.Detector(sift.CudaSiftConfig(col_width=752, row_width=480, numFeatures=5000, upscale=False), device=0)
    c = d.capacities()
    sum_px = sum(d.octave_dims(o)[0] * d.octave_dims(o)[1] for o in range(d.nOctaves))
    assert c["results"] == 6250
    assert c["candidates"] == max(16384, min(sum_px * 3 // 8, 1 << 20))
    assert c["refined"] == min(c["candidates"], 1 << 18) and c["oriented"] == 2 * c["refined"]
    d2 = sift.Detector(sift.CudaSiftConfig(col_width=752, row_width=480, numFeatures=5000, maxKeypoints=777), device=0)
    assert d2.capacities()["results"] == 777
    d3 = sift.Detector(sift.CudaSiftConfig(col_width=1920, row_width=1200, numFeatures=0, upscale=True), device=0)
    c3 = d3.capacities()
    assert 4096 <= c3["results"] <= 65536 and c3["candidates"] <= 1 << 20 and c3["oriented"] <= 1 << 19


def test_descriptor_mode_host_logic(sift):
    """sift_hip_set_descriptor_mode: two modes, set before warm-up (host-only)."""
    L = sift.lib()
    h = ctypes.c_void_p()
    c = sift._Config()
    L.sift_hip_default_config(ctypes.byref(c), 64, 64)
    assert L.sift_hip_create(ctypes.byref(c), 0, ctypes.byref(h)) == 0
    try:
        m = ctypes.c_int(-1)
        assert L.sift_hip_descriptor_mode(h, ctypes.byref(m)) == 0 and m.value == sift.SIFT_HIP_DESC_FAST
        assert L.sift_hip_set_descriptor_mode(h, 2) == -1
        assert L.sift_hip_set_descriptor_mode(h, sift.SIFT_HIP_DESC_EXACT) == 0
        assert L.sift_hip_descriptor_mode(h, ctypes.byref(m)) == 0 and m.value == sift.SIFT_HIP_DESC_EXACT
        assert L.sift_hip_set_descriptor_mode(h, sift.SIFT_HIP_DESC_FAST) == 0
    finally:
        L.sift_hip_destroy(h)
    assert L.sift_hip_set_descriptor_mode(None, 0) == -1
    d = sift.Detector(sift.CudaSiftConfig(col_width=64, row_width=64), device=0, exact_descriptors=True)
    assert d.exact_descriptors

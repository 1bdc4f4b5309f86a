"""ctypes binding of the CPU oracle (oracle/_build/libsift_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / baseline, never as the
thing measured or shipped.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# SIFT_ORACLE_BUILD=_build_asan: the sanitizer build (oracle/Makefile asan,
# tests/test_asan.py); default: the optimised build.
BUILD_DIR = os.environ.get("SIFT_ORACLE_BUILD", "_build")
ORACLE_LIB = os.path.join(ORACLE_DIR, BUILD_DIR, "libsift_oracle.so")
# Builds of the same restatement (oracle/Makefile): "pinned" is the parity pin
# of the HIP path; the others model OpenCV's AVX2 / AVX-512 dispatch as GCC
# compiles it (the ensemble the stated OpenCV tolerance comes from).
VARIANTS = {
    "pinned": ORACLE_LIB,
    "avx2-fma": os.path.join(ORACLE_DIR, "_build", "libsift_oracle_avx2fma.so"),
    "avx512-fma": os.path.join(ORACLE_DIR, "_build", "libsift_oracle_avx512fma.so"),
}


class Params(ctypes.Structure):
    _fields_ = [
        ("nfeatures", ctypes.c_int),
        ("nOctaveLayers", ctypes.c_int),
        ("contrastThreshold", ctypes.c_double),
        ("edgeThreshold", ctypes.c_double),
        ("sigma", ctypes.c_double),
        ("firstOctave", ctypes.c_int),
        ("nOctaves", ctypes.c_int),
    ]


class Kpt(ctypes.Structure):
    _fields_ = [
        ("x", ctypes.c_float),
        ("y", ctypes.c_float),
        ("size", ctypes.c_float),
        ("angle", ctypes.c_float),
        ("response", ctypes.c_float),
        ("octave", ctypes.c_int),
    ]


KPT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"), ("octave", "<i4")])

_libs = {}


def lib(variant: str = "pinned") -> ctypes.CDLL:
    if variant not in _libs:
        path = VARIANTS[variant]
        if not os.path.exists(path):
            subprocess.run(["make", "-C", ORACLE_DIR] + (["asan"] if BUILD_DIR == "_build_asan" else []), check=True,
                           capture_output=True)
        L = ctypes.CDLL(path)
        vp, i, l, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_double
        P = ctypes.POINTER(Params)
        L.sift_oracle_default_params.argtypes = [P]
        L.sift_oracle_gaussian_taps.argtypes = [d, vp, i]
        L.sift_oracle_gaussian_taps.restype = i
        L.sift_oracle_num_octaves.argtypes = [i, i, P]
        L.sift_oracle_num_octaves.restype = i
        L.sift_oracle_octave_dims.argtypes = [i, i, P, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        L.sift_oracle_gaussian_pyramid.argtypes = [vp, i, i, P, vp]
        L.sift_oracle_gaussian_pyramid.restype = l
        L.sift_oracle_extrema.argtypes = [vp, i, i, P, vp, l]
        L.sift_oracle_extrema.restype = l
        L.sift_oracle_detect_and_compute.argtypes = [vp, i, i, P, i, vp, vp, l]
        L.sift_oracle_detect_and_compute.restype = l
        if hasattr(L, "sift_oracle_stage_ms"):
            L.sift_oracle_stage_ms.argtypes = [vp, i]
            L.sift_oracle_stage_ms.restype = i
        L.sift_oracle_compute_descriptors.argtypes = [vp, i, i, P, vp, l, vp]
        L.sift_oracle_knn2.argtypes = [vp, l, vp, l, i, vp, vp]
        L.sift_oracle_variant.restype = ctypes.c_char_p
        got = L.sift_oracle_variant().decode()
        if got != variant:
            raise RuntimeError(f"{path} is the {got!r} build, expected {variant!r}")
        _libs[variant] = L
    return _libs[variant]


def params(nfeatures=0, nOctaveLayers=3, contrastThreshold=0.04, edgeThreshold=10.0, sigma=1.6, firstOctave=-1, nOctaves=0) -> Params:
    p = Params()
    lib().sift_oracle_default_params(ctypes.byref(p))
    p.nfeatures, p.nOctaveLayers, p.contrastThreshold = nfeatures, nOctaveLayers, contrastThreshold
    p.edgeThreshold, p.sigma, p.firstOctave, p.nOctaves = edgeThreshold, sigma, firstOctave, nOctaves
    return p


def from_config(cfg) -> Params:
    """Oracle parameters equivalent to a sift_amd.CudaSiftConfig."""
    return params(cfg.numFeatures, cfg.numOctaveLayers, cfg.contrastThreshould, cfg.edgeThreshould, cfg.sigma,
                  -1 if cfg.upscale else 0, cfg.numOctaves)


def gaussian_taps(sigma: float) -> np.ndarray:
    buf = np.zeros(128, np.float32)
    n = lib().sift_oracle_gaussian_taps(sigma, buf.ctypes.data, 128)
    return buf[:n].copy()


def num_octaves(w: int, h: int, p: Params) -> int:
    return lib().sift_oracle_num_octaves(w, h, ctypes.byref(p))


def octave_dims(w: int, h: int, p: Params, o: int):
    ow, oh = ctypes.c_int(), ctypes.c_int()
    lib().sift_oracle_octave_dims(w, h, ctypes.byref(p), o, ctypes.byref(ow), ctypes.byref(oh))
    return ow.value, oh.value


def gaussian_pyramid(img: np.ndarray, p: Params):
    """List (per octave) of arrays (L+3, oh, ow)."""
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape
    n = lib().sift_oracle_gaussian_pyramid(img.ctypes.data, w, h, ctypes.byref(p), None)
    buf = np.zeros(n, np.float32)
    lib().sift_oracle_gaussian_pyramid(img.ctypes.data, w, h, ctypes.byref(p), buf.ctypes.data)
    out, off = [], 0
    L = p.nOctaveLayers
    for o in range(num_octaves(w, h, p)):
        ow, oh = octave_dims(w, h, p, o)
        cnt = ow * oh * (L + 3)
        out.append(buf[off:off + cnt].reshape(L + 3, oh, ow))
        off += cnt
    return out


def extrema(img: np.ndarray, p: Params, variant: str = "pinned") -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape
    n = lib(variant).sift_oracle_extrema(img.ctypes.data, w, h, ctypes.byref(p), None, 0)
    q = np.zeros((max(n, 1), 4), np.int32)
    lib(variant).sift_oracle_extrema(img.ctypes.data, w, h, ctypes.byref(p), q.ctypes.data, n)
    return q[:n]


def detect_and_compute(img: np.ndarray, p: Params, threads: int = 0, cap: int = 1 << 20, variant: str = "pinned"):
    """(keypoints structured array, descriptors float32 (n,128) of 0..255 integers)."""
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape
    kp = np.zeros(cap, KPT_DTYPE)
    desc = np.zeros((cap, 128), np.float32)
    n = lib(variant).sift_oracle_detect_and_compute(img.ctypes.data, w, h, ctypes.byref(p), threads, kp.ctypes.data,
                                                    desc.ctypes.data, cap)
    n = min(n, cap)
    return kp[:n].copy(), desc[:n].copy()


def compute_descriptors(img: np.ndarray, p: Params, kpts: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    h, w = img.shape
    k = np.ascontiguousarray(kpts.astype(KPT_DTYPE))
    desc = np.zeros((len(k), 128), np.float32)
    lib().sift_oracle_compute_descriptors(img.ctypes.data, w, h, ctypes.byref(p), k.ctypes.data, len(k), desc.ctypes.data)
    return desc


def knn2(query: np.ndarray, train: np.ndarray, threads: int = 0):
    q = np.ascontiguousarray(query, np.float32)
    t = np.ascontiguousarray(train, np.float32)
    idx = np.zeros((len(q), 2), np.int32)
    dist = np.zeros((len(q), 2), np.float32)
    lib().sift_oracle_knn2(q.ctypes.data, len(q), t.ctypes.data, len(t), threads, idx.ctypes.data, dist.ctypes.data)
    return idx, dist


STAGES = ("initial", "pyramid", "dog", "candidates", "keypoints", "descriptors")


def stage_ms(variant: str = "pinned") -> dict:
    """Wall time per stage (ms) of the last detect_and_compute call of this build."""
    out = np.zeros(6, np.float64)
    lib(variant).sift_oracle_stage_ms(out.ctypes.data, 6)
    return dict(zip(STAGES, (round(float(x), 3) for x in out)))

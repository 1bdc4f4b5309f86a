"""CPU oracle (oracle/sift_oracle.cpp) checks -- no GPU.

The oracle restates OpenCV 4.x SIFT; OpenCV is absent here and
the reference ships no golden vectors, so OpenCV parity is UNPINNED.  What is
pinned here:
  * regression: the committed fixtures tests/golden/camera256.npz + golden.json
    (made by tests/golden/make_golden.py) reproduce bit for bit;
  * the algorithm's own invariants, recomputed independently in numpy: tap
    construction, octave geometry, nearest-neighbour decimation, the DoG 3x3x3
    extremum test, descriptor normalisation, brute-force knn-2.
"""
import json
import math
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "camera256.npz"), allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    with open(os.path.join(GOLD, "golden.json")) as f:
        meta = json.load(f)
    return data, meta


@pytest.fixture(scope="module")
def camera(gold):
    return gold[0]["camera256"].astype(np.float32)


def sha(a):
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# --------------------------------------------------------------- fixtures ----

def test_golden_taps(oracle, gold):
    data, meta = gold
    for s in meta["sigmas"]:
        assert np.array_equal(oracle.gaussian_taps(s).view(np.uint32), data[f"taps_{s!r}"].view(np.uint32)), s


@pytest.mark.parametrize("name", ["default", "base_n60"])
def test_golden_pyramid(oracle, gold, camera, name):
    data, meta = gold
    pyr = oracle.gaussian_pyramid(camera, oracle.params(**meta["configs"][name]))
    got = [[sha(pl) for pl in planes] for planes in pyr]
    assert got == meta["pyramid_sha"][name]


@pytest.mark.parametrize("name", ["default", "base_n60"])
def test_golden_extrema_keypoints_descriptors(oracle, gold, camera, name):
    data, meta = gold
    p = oracle.params(**meta["configs"][name])
    assert np.array_equal(oracle.extrema(camera, p), data[f"{name}_extrema"])
    k, d = oracle.detect_and_compute(camera, p, threads=4)
    gk = data[f"{name}_kpts"]
    assert len(k) == len(gk) and len(k) > 50
    for f in gk.dtype.names:
        assert np.array_equal(k[f].view(np.uint32), gk[f].view(np.uint32)), f
    assert np.array_equal(d.astype(np.uint8), data[f"{name}_desc"])


def test_golden_rot90_match(oracle, gold, camera):
    data, _ = gold
    p = oracle.params()
    _, da = oracle.detect_and_compute(camera, p, threads=4)
    _, db = oracle.detect_and_compute(np.ascontiguousarray(np.rot90(camera)), p, threads=4)
    idx, dist = oracle.knn2(da, db, threads=4)
    assert np.array_equal(idx, data["rot90_knn_idx"])
    assert np.array_equal(dist.view(np.uint32), data["rot90_knn_dist"].view(np.uint32))
    # SIFT is rotation invariant: most keypoints find their rotated twin.
    good = dist[:, 0] < 0.8 * dist[:, 1]
    assert good.mean() > 0.7


def test_golden_synth_frames(sift, gold):
    _, meta = gold
    for key, h in meta["synth_sha"].items():
        seed, wh = key.split("_")
        w, hh = map(int, wh.split("x"))
        img = sift.synth_frame(int(seed), w, hh)
        assert img.dtype == np.float32 and img.shape == (hh, w)
        assert np.all(img == np.round(img)) and img.min() >= 0 and img.max() <= 255
        assert sha(img) == h, key


# ------------------------------------------------------------- invariants ----

@pytest.mark.parametrize("sigma", [0.5, 1.0, 1.2262735, 1.6, 2.4525471, 3.0900346, 5.0])
def test_taps_recipe(oracle, sigma):
    """getGaussianKernel for CV_32F: ksize = cvRound(8 sigma + 1) | 1, exp in double, normalised, cast."""
    t = oracle.gaussian_taps(sigma)
    n = int(math.floor(sigma * 8 + 1 + 0.5)) | 1
    assert len(t) == n
    assert np.array_equal(t, t[::-1])
    x = np.arange(n) - (n - 1) / 2
    ref = np.exp(-x * x / (2 * sigma * sigma))
    ref = (ref / ref.sum()).astype(np.float32)
    assert np.abs(t.astype(np.float64) - ref).max() <= 2 * np.finfo(np.float32).eps * ref.max()
    assert abs(float(t.astype(np.float64).sum()) - 1.0) < 1e-6


@pytest.mark.parametrize("w,h,first", [(1920, 1200, 0), (1920, 1200, -1), (752, 480, -1), (257, 191, 0), (64, 48, -1)])
def test_octave_geometry(oracle, w, h, first):
    p = oracle.params(firstOctave=first)
    n = oracle.num_octaves(w, h, p)
    bw, bh = (2 * w, 2 * h) if first < 0 else (w, h)
    assert n == int(math.floor(math.log2(min(bw, bh)) - 2 + 0.5)) - first
    dims = [oracle.octave_dims(w, h, p, o) for o in range(n)]
    assert dims[0] == (bw, bh)
    for a, b in zip(dims, dims[1:]):
        assert b == (a[0] // 2, a[1] // 2)


def test_pyramid_decimation_and_blur_invariants(oracle, camera):
    p = oracle.params()
    pyr = oracle.gaussian_pyramid(camera, p)
    L = p.nOctaveLayers
    for o in range(1, len(pyr)):
        prev, cur = pyr[o - 1], pyr[o]
        dec = prev[L][: 2 * cur.shape[1]: 2, : 2 * cur.shape[2]: 2]
        assert np.array_equal(cur[0], dec)  # INTER_NEAREST 2x decimation of layer L
    for planes in pyr:  # blurs are convex combinations: range can only shrink
        for pl in planes:
            assert pl.min() >= -1e-3 and pl.max() <= 255 + 1e-3


def test_extrema_are_3x3x3_extrema(oracle, camera):
    """Every candidate passes OpenCV's test; a numpy scan finds exactly the same set."""
    p = oracle.params(firstOctave=0)
    pyr = oracle.gaussian_pyramid(camera, p)
    cand = oracle.extrema(camera, p)
    L, border = p.nOctaveLayers, 5
    thr = math.floor(0.5 * p.contrastThreshold / L * 255)
    found = []
    for o, g in enumerate(pyr):
        dog = g[1:] - g[:-1]  # float32 subtraction, as OpenCV's subtract
        H, W = dog.shape[1:]
        if H <= 2 * border or W <= 2 * border:
            continue
        for layer in range(1, L + 1):
            c = dog[layer, border:H - border, border:W - border]
            nb = np.stack([dog[layer + dl, border + dy:H - border + dy, border + dx:W - border + dx]
                           for dl in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                           if (dl, dy, dx) != (0, 0, 0)])
            pos = (c > 0) & np.all(c >= nb, axis=0)
            neg = (c < 0) & np.all(c <= nb, axis=0)
            rr, cc = np.nonzero((np.abs(c) > thr) & (pos | neg))
            found += [(o, layer, r + border, q + border) for r, q in zip(rr, cc)]
    got = sorted(map(tuple, cand.tolist()))
    assert got == sorted(found)
    assert len(got) > 100


def test_descriptor_invariants(oracle, camera):
    k, d = oracle.detect_and_compute(camera, oracle.params(), threads=4)
    assert d.shape == (len(k), 128)
    assert np.all(d == np.round(d)) and d.min() >= 0 and d.max() <= 255
    n = np.linalg.norm(d.astype(np.float64), axis=1)
    assert np.all(np.abs(n - 512) < 512 * 0.02)  # unit norm x 512 after clip + renorm, rounded
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360)) and np.all(k["size"] > 0)
    assert np.all(k["response"] > 0)
    octv = k["octave"] & 255
    octv = np.where(octv >= 128, octv - 256, octv)
    assert octv.min() >= -1 and np.all(((k["octave"] >> 8) & 255) >= 1)


def test_compute_matches_detect(oracle, camera):
    p = oracle.params()
    k, d = oracle.detect_and_compute(camera, p, threads=4)
    d2 = oracle.compute_descriptors(camera, p, k)
    assert np.array_equal(d, d2)


def test_thread_count_invariance(oracle, sift):
    img = sift.synth_frame(5, 320, 240)
    p = oracle.params(nfeatures=150)
    k1, d1 = oracle.detect_and_compute(img, p, threads=1)
    k8, d8 = oracle.detect_and_compute(img, p, threads=8)
    assert np.array_equal(k1, k8) and np.array_equal(d1, d8)


def test_knn2_bruteforce(oracle):
    rng = np.random.default_rng(3)
    q = rng.integers(0, 40, (300, 128)).astype(np.float32)
    t = rng.integers(0, 40, (257, 128)).astype(np.float32)
    t[17] = t[5]  # duplicate train rows: ties break to the lower index
    q[:4] = t[5]
    idx, dist = oracle.knn2(q, t, threads=4)
    d2 = ((q[:, None, :].astype(np.int64) - t[None, :, :].astype(np.int64)) ** 2).sum(-1)
    order = np.lexsort((np.broadcast_to(np.arange(len(t)), d2.shape), d2), axis=1)
    assert np.array_equal(idx, order[:, :2].astype(np.int32))
    best = np.take_along_axis(d2, order[:, :2], 1)
    assert np.allclose(dist.astype(np.float64) ** 2, best, rtol=1e-6, atol=1e-3)
    assert np.all(idx[:4, 0] == 5) and np.all(idx[:4, 1] == 17)


def test_blank_and_tiny_images(oracle):
    p = oracle.params()
    k, d = oracle.detect_and_compute(np.zeros((64, 80), np.float32), p, threads=2)
    assert len(k) == 0 and d.shape == (0, 128)
    k, d = oracle.detect_and_compute(np.full((16, 16), 77, np.float32), p, threads=2)
    assert len(k) == 0

"""GPU path (C ABI) against the committed golden fixtures (tests/golden/).

Same bar as test_gpu_parity.py: keypoints bit-exact, descriptors |diff| <= 1
with >= 99.8 % exact (parity_bar.py), pyramid planes bit-exact (sha256 per plane).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from test_gpu_parity import assert_same_keypoints, gpu_keypoints, sort_keys
from parity_bar import assert_descriptor_bar

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gold():
    with np.load(os.path.join(GOLD, "camera256.npz"), allow_pickle=False) as z:
        data = {k: z[k] for k in z.files}
    with open(os.path.join(GOLD, "golden.json")) as f:
        return data, json.load(f)


def config_for(sift, meta_cfg):
    return sift.CudaSiftConfig(col_width=256, row_width=256, upscale=meta_cfg.get("firstOctave", -1) < 0,
                               numFeatures=meta_cfg.get("nfeatures", 0), numOctaves=0)


@pytest.mark.parametrize("name", ["default", "base_n60"])
def test_camera_golden(sift, gold, name):
    data, meta = gold
    img = data["camera256"].astype(np.float32)
    det = sift.Detector(config_for(sift, meta["configs"][name]))
    det.gpuWarmUpAndAllocate()
    det.detectAndCompute(img)
    shas = meta["pyramid_sha"][name]
    assert det.nOctaves == len(shas)
    for o, planes in enumerate(shas):
        for layer, h in enumerate(planes):
            g = np.ascontiguousarray(det.debug_gaussian(o, layer))
            assert hashlib.sha256(g.tobytes()).hexdigest() == h, (o, layer)
    cand = det.debug_candidates()
    ref = data[f"{name}_extrema"]
    assert np.array_equal(cand[np.lexsort(cand.T[::-1])], ref[np.lexsort(ref.T[::-1])])
    gk, gd, _ = gpu_keypoints(det)
    ok, od = data[f"{name}_kpts"], data[f"{name}_desc"].astype(np.float32)
    assert_same_keypoints(gk, ok)
    assert_descriptor_bar(gd[sort_keys(gk)], od[sort_keys(ok)], "golden")


def test_camera_rot90_match(sift, oracle, gold):
    """HIP matcher on HIP descriptors of the crop and its 90-degree rotation:
    top-2 exact against the oracle's knn on the same descriptors, and the
    ratio-test match count within 2 % of the golden (oracle-descriptor) one."""
    data, _ = gold
    img = data["camera256"].astype(np.float32)
    cfg = sift.CudaSiftConfig(col_width=256, row_width=256, upscale=True, numFeatures=0)
    descs = []
    for im in (img, np.ascontiguousarray(np.rot90(img))):
        det = sift.Detector(cfg)
        det.gpuWarmUpAndAllocate()
        det.detectAndCompute(im)
        _, d, _ = gpu_keypoints(det)
        descs.append(d)
    da, db = descs
    nq, nt = len(da), len(db)
    dq = sift.DeviceArray.from_numpy(da.astype(np.float16))
    dt = sift.DeviceArray.from_numpy(db.astype(np.float16))
    idx2, d2 = sift.DeviceArray(nq * 8), sift.DeviceArray(nq * 8)
    sift.Matcher(nq, nt).match_device(dq.value, nq, dt.value, nt, 0.8, False, idx2.value, d2.value)
    gi, gd = idx2.to_numpy(np.int32, (nq, 2)), d2.to_numpy(np.float32, (nq, 2))
    oi, od = oracle.knn2(da, db)
    assert np.array_equal(gi, oi)
    assert np.array_equal(np.sqrt(gd).astype(np.float32), od)
    ref = data["rot90_knn_dist"]
    n_gpu = int((od[:, 0] < 0.8 * od[:, 1]).sum())
    n_ref = int((ref[:, 0] < 0.8 * ref[:, 1]).sum())
    assert nq == len(ref) and abs(n_gpu - n_ref) <= 0.02 * n_ref, (n_gpu, n_ref)


@pytest.mark.parametrize("name", ["default", "base_n60"])
def test_camera_golden_exact_descriptors(sift, gold, name):
    """Exact descriptor mode (SIFT_HIP_DESC_EXACT): the golden fixture's uint8
    descriptors byte for byte."""
    data, meta = gold
    img = data["camera256"].astype(np.float32)
    det = sift.Detector(config_for(sift, meta["configs"][name]), exact_descriptors=True)
    det.gpuWarmUpAndAllocate()
    det.detectAndCompute(img)
    gk, gd, _ = gpu_keypoints(det)
    ok, od = data[f"{name}_kpts"], data[f"{name}_desc"].astype(np.float32)
    assert_same_keypoints(gk, ok)
    assert np.array_equal(gd[sort_keys(gk)], od[sort_keys(ok)])


def test_camera_rot90_match_exact(sift, gold):
    """Exact descriptors of the crop and its rotation through the HIP matcher:
    the golden knn-2 distances (oracle descriptors, oracle matcher) exactly."""
    data, _ = gold
    img = data["camera256"].astype(np.float32)
    cfg = sift.CudaSiftConfig(col_width=256, row_width=256, upscale=True, numFeatures=0)
    descs, keys = [], []
    for im in (img, np.ascontiguousarray(np.rot90(img))):
        det = sift.Detector(cfg, exact_descriptors=True)
        det.gpuWarmUpAndAllocate()
        det.detectAndCompute(im)
        gk, d, _ = gpu_keypoints(det)
        descs.append(d)
        keys.append(gk)
    da, db = descs
    nq, nt = len(da), len(db)
    dq = sift.DeviceArray.from_numpy(da.astype(np.float16))
    dt = sift.DeviceArray.from_numpy(db.astype(np.float16))
    idx2, d2 = sift.DeviceArray(nq * 8), sift.DeviceArray(nq * 8)
    sift.Matcher(nq, nt).match_device(dq.value, nq, dt.value, nt, 0.8, False, idx2.value, d2.value)
    gd = d2.to_numpy(np.float32, (nq, 2))
    ref, ok = data["rot90_knn_dist"], data["default_kpts"]  # the golden's queries: the "default" config's keypoints
    assert nq == len(ref) == len(ok)
    # a query's distances depend on its descriptor and the train set only: compare in keypoint order
    assert np.array_equal(np.sqrt(gd).astype(np.float32)[sort_keys(keys[0])], ref[sort_keys(ok)])

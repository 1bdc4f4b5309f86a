"""GPU input path: 8-bit frames, pipelined submit/wait.

Bar: an 8-bit frame gives exactly (bit for bit) the keypoints, features and
descriptors of the float frame holding the same values -- OpenCV converts
CV_8U input to float exactly -- and a frame submitted through the pipelined
path gives exactly what the synchronous call gives, with prev_descriptor = the
previous frame's descriptors.  The float path itself is held to the oracle by
test_gpu_parity.py; the non-default-sigma case (8-bit conversion fallback) is
also checked against the oracle here.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_same_keypoints, gpu_keypoints, make_detector, sort_keys
from parity_bar import assert_descriptor_bar

pytestmark = pytest.mark.gpu


def results(det):
    det.copyToHost(True)
    return det.final_kpts.copy(), det.final_features.copy(), det.descriptors.view(np.uint16).copy()


def assert_identical(a, b):
    for x, y in zip(a, b):
        assert x.shape == y.shape and np.array_equal(x.view(np.uint32) if x.dtype == np.float32 else x,
                                                     y.view(np.uint32) if y.dtype == np.float32 else y)


@pytest.mark.parametrize("w,h,upscale,nOct,nfeat,frame,sigma", [
    (1920, 1200, False, 3, 5000, 0, 1.6),   # C2 bench workload: fused 8-bit first blur (13 taps)
    (257, 191, True, 0, 0, 2, 1.6),         # doubled base: 8-bit upsample
    (300, 200, False, 0, 0, 5, 2.0),        # other init radius: conversion kernel + float blur
])
def test_u8_equals_f32(sift, w, h, upscale, nOct, nfeat, frame, sigma):
    img = sift.synth_frame(frame, w, h)
    _, det = make_detector(sift, w, h, upscale=upscale, numOctaves=nOct, numFeatures=nfeat, sigma=sigma)
    det.detectAndCompute(img)
    ref = results(det)
    assert len(ref[0]) > 20
    det.detectAndCompute(img.astype(np.uint8))
    assert_identical(results(det), ref)


def test_u8_other_sigma_vs_oracle(sift, oracle):
    w, h = 300, 200
    img = sift.synth_frame(5, w, h)
    cfg, det = make_detector(sift, w, h, sigma=2.0, numFeatures=0)
    det.detectAndCompute(img.astype(np.uint8))
    gk, gd, _ = gpu_keypoints(det)
    ok, od = oracle.detect_and_compute(img, oracle.from_config(cfg))
    assert_same_keypoints(gk, ok)
    assert_descriptor_bar(gd[sort_keys(gk)], od[sort_keys(ok)], "u8 sigma 2")


def test_u8_device_and_strided_host(sift):
    w, h = 640, 360
    img = sift.synth_frame(3, w, h)
    _, det = make_detector(sift, w, h, upscale=True, numFeatures=500)
    det.detectAndCompute(img)
    ref = results(det)
    # strided 8-bit host frame (a view into a wider buffer)
    wide = np.zeros((h, w + 37), np.uint8)
    wide[:, 5:5 + w] = img.astype(np.uint8)
    det.detectAndCompute(wide[:, 5:5 + w])
    assert_identical(results(det), ref)
    # 8-bit frame already in device memory, row stride 704 bytes
    pitch = 704
    host = np.zeros((h, pitch), np.uint8)
    host[:, :w] = img.astype(np.uint8)
    dev = sift.DeviceArray.from_numpy(host)
    det.detectAndComputeDevice(dev.value, pitch, u8=True)
    assert_identical(results(det), ref)


def test_pipelined_equals_sync(sift):
    w, h = 752, 480
    frames = [sift.synth_frame(30 + i, w, h) for i in range(7)]
    _, det = make_detector(sift, w, h, numFeatures=2000)
    sync = []
    for f in frames:
        det.detectAndCompute(f)
        sync.append(results(det))
    _, pdet = make_detector(sift, w, h, numFeatures=2000)
    # frame i+1 submitted before frame i is waited (two in flight past the
    # current one); formats alternate
    fmt = lambda i, f: f.astype(np.uint8) if i % 2 else f
    tickets = [pdet.submit(fmt(0, frames[0]))]
    for i in range(len(frames)):
        if i + 1 < len(frames):
            tickets.append(pdet.submit(fmt(i + 1, frames[i + 1])))
        pdet.wait(tickets[i])
        got = results(pdet)
        assert_identical(got, sync[i])
        if i > 0:
            n = len(sync[i - 1][0])
            assert pdet.prev_size == n
            prev = np.empty((n, 128), np.uint16)
            sift._check(sift.lib().sift_hip_memcpy_d2h(prev.ctypes.data, pdet.prev_descriptor.data(), prev.nbytes), "d2h")
            assert np.array_equal(prev, sync[i - 1][2])
        else:
            assert pdet.prev_size == 0


def test_pipeline_limits(sift):
    w, h = 128, 96
    img = sift.synth_frame(1, w, h)
    _, det = make_detector(sift, w, h, lanes=1)  # one lane: two frames past the current one
    t0, t1 = det.submit(img), det.submit(img)
    with pytest.raises(sift.SiftHipError):  # a third frame past the current one
        det.submit(img)
    with pytest.raises(sift.SiftHipError):  # never submitted
        det.wait(t1 + 5)
    det.wait(t1)
    det.wait(t0)  # still held: frames current-1 .. current+2 never share a slot
    t2 = det.submit(img.astype(np.uint8))
    det.wait(t2)
    with pytest.raises(sift.SiftHipError):
        det.submit(np.zeros((h, w), np.int16).astype(np.float32)[:, :-1])

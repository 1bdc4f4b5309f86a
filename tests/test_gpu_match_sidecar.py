"""Matcher sidecars (sift_hip_matcher_set_sidecars): descriptor buffers a
detector hands out carry int8 codes + key biases written by the descriptor
kernel, and a single pair of such buffers is matched from them directly
(k_match_direct, no fp16 conversion).  Bar: top-2 indices, squared distances
and ratio-test matches identical to the converting path and to the oracle's
knn-2 (exact integers), for full and ragged row counts, both descriptor modes,
batch-handle frames and single-frame handles; matchBruteForce on
prev_descriptor / device_descriptor (the reference's call,
/root/reference/tool/extract_and_match_example.cc:87) takes this path.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def run(sift, m, qp, nq, tp, nt, squared=False):
    idx2, d2, mt = sift.DeviceArray(nq * 8), sift.DeviceArray(nq * 8), sift.DeviceArray(nq * 4)
    m.match_device(qp, nq, tp, nt, 0.8, squared, idx2.value, d2.value, mt.value)
    return idx2.to_numpy(np.int32, (nq, 2)), d2.to_numpy(np.float32, (nq, 2)), mt.to_numpy(np.int32, (nq,))


def host_desc(sift, ptr, n):
    out = np.empty((n, 128), np.uint16)
    sift._check(sift.lib().sift_hip_memcpy_d2h(out.ctypes.data, ptr, out.nbytes), "d2h")
    return out.view(np.float16).astype(np.float32)


@pytest.mark.parametrize("exact", [False, True])
def test_sidecar_pair_equals_converted_and_oracle(sift, oracle, exact):
    w, h = 1920, 1200
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numOctaves=3, numFeatures=2000)
    det = sift.Detector(cfg, exact_descriptors=exact)
    det.gpuWarmUpAndAllocate()
    det.detectAndCompute(sift.synth_frame(77, w, h))
    det.detectAndCompute(sift.synth_frame(78, w, h))
    n0, n1 = det.prev_size, det.total_size
    assert n0 >= 2000 and n1 >= 2000
    q, t = det.prev_descriptor.data(), det.device_descriptor.data()
    dq, dt = host_desc(sift, q, n0), host_desc(sift, t, n1)
    m = sift.Matcher(max(n0, n1), max(n0, n1))
    mc = sift.Matcher(max(n0, n1), max(n0, n1))
    mc.set_sidecars(False)
    for nq, nt in [(2000, 2000), (n0, n1), (1, n1), (n0, 1), (257, 1999), (1500, 300)]:
        a = run(sift, m, q, nq, t, nt)
        b = run(sift, mc, q, nq, t, nt)
        for x, y in zip(a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), (nq, nt)
        oi, od = oracle.knn2(dq[:nq], dt[:nt])
        assert np.array_equal(a[0], oi), (nq, nt)
        valid = oi >= 0
        assert np.array_equal(np.sqrt(a[1][valid]).astype(np.float32), od[valid]), (nq, nt)
    # the reference's call: matchBruteForce(prev_descriptor, n0, device_descriptor, n1), squared ratio
    mb = sift.matchBruteForce(det.prev_descriptor, n0, det.device_descriptor, n1)
    assert np.array_equal(mb, run(sift, mc, q, n0, t, n1, squared=True)[2])


def test_sidecar_batch_frames_and_foreign_buffers(sift, oracle):
    """Frames of a batch handle (each results slot at its frame's arena) and a
    pairing of a detector buffer with a foreign one (converted path)."""
    import torch

    w, h = 752, 480
    B = 4
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, upscale=True, numFeatures=0)
    det = sift.Detector(cfg, batch=B)
    det.gpuWarmUpAndAllocate()
    frames = torch.from_numpy(np.stack([sift.synth_frame(20 + i, w, h) for i in range(B)])).cuda()
    torch.cuda.synchronize()
    det.detectBatchDevice(frames.data_ptr(), B, w * 4, w * h * 4)
    res = [det.batch_results(i) for i in range(B)]
    m = sift.Matcher(4096, 4096)
    for i in range(B - 1):
        (n0, _, _, _, p0), (n1, _, _, _, p1) = res[i], res[i + 1]
        d0, d1 = host_desc(sift, p0, n0), host_desc(sift, p1, n1)
        gi, gd, _ = run(sift, m, p0, n0, p1, n1)
        oi, od = oracle.knn2(d0, d1)
        assert np.array_equal(gi, oi), i
        foreign = sift.DeviceArray.from_numpy(np.ascontiguousarray(d1.astype(np.float16)).view(np.uint16))
        fi, fd, _ = run(sift, m, p0, n0, foreign.value, n1)
        assert np.array_equal(fi, oi) and np.array_equal(fd.view(np.uint32), gd.view(np.uint32)), i


def test_sidecar_micro_batch_frames(sift):
    """Micro-batched device frames (frame i of a launch group in arena i):
    prev_descriptor x device_descriptor inside a group and across groups match
    from the sidecars exactly as the converting path does."""
    import torch

    w, h = 752, 480
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=2000)
    det = sift.Detector(cfg, lanes=2, micro_batch=3)
    det.gpuWarmUpAndAllocate()
    dev = [torch.from_numpy(sift.synth_frame(120 + i, w, h)).cuda() for i in range(7)]
    torch.cuda.synchronize()
    tickets = [det.submitDevice(d.data_ptr(), w * 4) for d in dev]
    m = sift.Matcher(4096, 4096)
    mc = sift.Matcher(4096, 4096)
    mc.set_sidecars(False)
    for t in tickets[1:]:  # frames 1, 2 share a group with their predecessor; 3 and 6 start groups
        det.wait(t)
        n0, n1 = det.prev_size, det.total_size
        assert n0 > 100 and n1 > 100
        a = run(sift, m, det.prev_descriptor.data(), n0, det.device_descriptor.data(), n1)
        b = run(sift, mc, det.prev_descriptor.data(), n0, det.device_descriptor.data(), n1)
        for x, y in zip(a, b):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), t

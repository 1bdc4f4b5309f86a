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


def test_written_rows_drop_the_sidecar(sift, oracle):
    """(Round-5 review item 7.)  A caller that writes into a detector's
    descriptor rows through the writable view (DeviceBuffer.mutable_data ->
    sift_hip_descriptors_written) gets the converting path's results on those
    rows -- the stale int8 codes are never matched -- and the sidecar is valid
    again once the detector writes that buffer with a new frame."""
    w, h = 752, 480
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=2000)
    det = sift.Detector(cfg, lanes=1)
    det.gpuWarmUpAndAllocate()
    det.detectAndCompute(sift.synth_frame(90, w, h))
    det.detectAndCompute(sift.synth_frame(91, w, h))
    n0, n1 = det.prev_size, det.total_size
    q, t = det.prev_descriptor.data(), det.device_descriptor.data()
    m = sift.Matcher(4096, 4096)
    mc = sift.Matcher(4096, 4096)
    mc.set_sidecars(False)
    before = run(sift, m, q, n0, t, n1)
    # Overwrite the current frame's rows: new integer descriptors (a permutation
    # of the rows and a shifted copy), as a caller post-processing them would.
    rows = host_desc(sift, t, n1)
    new = np.ascontiguousarray(np.clip(rows[::-1] + 3, 0, 255).astype(np.float16)).view(np.uint16)
    wp = det.device_descriptor.mutable_data()
    assert wp == t
    sift._check(sift.lib().sift_hip_memcpy_h2d(wp, new.ctypes.data, new.nbytes), "h2d")
    after = run(sift, m, q, n0, t, n1)
    conv = run(sift, mc, q, n0, t, n1)
    for x, y in zip(after, conv):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))
    oi, _ = oracle.knn2(host_desc(sift, q, n0), new.view(np.float16).astype(np.float32))
    assert np.array_equal(after[0], oi) and not np.array_equal(after[0], before[0])
    # New frames into the same slots (lanes=1: the four results slots come round) make the
    # sidecars valid again; the results stay the converting path's.
    for i in range(4):
        det.detectAndCompute(sift.synth_frame(92 + i, w, h))
    n0, n1 = det.prev_size, det.total_size
    a = run(sift, m, det.prev_descriptor.data(), n0, det.device_descriptor.data(), n1)
    b = run(sift, mc, det.prev_descriptor.data(), n0, det.device_descriptor.data(), n1)
    for x, y in zip(a, b):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_codes_batched_from_sidecars(sift, oracle):
    """sift_hip_match_codes_batched on code sets taken from detector sidecars
    (results_sidecar) and packed as multi.all_gather_codes lays them out:
    top-2 indices and d^2 equal the oracle's knn-2 on the fp16 rows; the
    sidecar codes equal multi.codes_from_rows of the rows."""
    import torch

    from sift_amd import multi

    w, h = 752, 480
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=2000)
    det = sift.Detector(cfg, lanes=1)
    det.gpuWarmUpAndAllocate()
    sets = []
    for f in (30, 31, 32):
        det.detectAndCompute(sift.synth_frame(f, w, h))
        n = det.total_size
        cp, kp = det.results_sidecar()
        codes = torch.empty((n, 128), dtype=torch.int8, device="cuda")
        keys = torch.empty(n, dtype=torch.int32, device="cuda")
        rows = torch.empty((n, 128), dtype=torch.int16, device="cuda")
        torch.cuda.synchronize()
        for dst, src, nb in ((codes, cp, n * 128), (keys, kp, n * 4), (rows, det.device_descriptor.data(), n * 256)):
            sift._check(sift.lib().sift_hip_memcpy_d2d(dst.data_ptr(), src, nb, None), "d2d")
        torch.cuda.synchronize()
        c2, k2 = multi.codes_from_rows(rows)
        assert torch.equal(c2, codes) and torch.equal(k2, keys)
        sets.append((codes, keys, rows, n))
    n_pad = multi.code_block_rows(max(s[3] for s in sets))
    buf = torch.cat([multi.pack_codes(c, k, n_pad) for c, k, _, _ in sets])
    pairs = []
    for a, b in ((0, 1), (1, 2), (2, 0), (0, 2)):
        qa, qk = multi.code_set(a, n_pad)
        ta, tk = multi.code_set(b, n_pad)
        pairs.append((qa, qk, sets[a][3], ta, tk, sets[b][3]))
    pairs.append(pairs[0][:5] + (300,))  # a ragged train set
    tot = sum(p[2] for p in pairs)
    idx2 = torch.empty((tot, 2), dtype=torch.int32, device="cuda")
    d2 = torch.empty((tot, 2), dtype=torch.float32, device="cuda")
    m = sift.Matcher(4096, 4096, max_pairs=8)
    m.match_codes_batched(buf.data_ptr(), buf.data_ptr(), pairs, idx2_ptr=idx2.data_ptr(), d2_ptr=d2.data_ptr())
    torch.cuda.synchronize()
    gi, gd = idx2.cpu().numpy(), d2.cpu().numpy()
    off = 0
    for (a, b), p in zip(((0, 1), (1, 2), (2, 0), (0, 2), (0, 1)), pairs):
        fq = sets[a][2].cpu().numpy().view(np.float16).astype(np.float32)
        ft = sets[b][2].cpu().numpy().view(np.float16).astype(np.float32)[: p[5]]
        oi, od = oracle.knn2(fq, ft)
        assert np.array_equal(gi[off: off + p[2]], oi), (a, b)
        valid = oi >= 0
        assert np.array_equal(np.sqrt(gd[off: off + p[2]][valid]).astype(np.float32), od[valid]), (a, b)
        off += p[2]

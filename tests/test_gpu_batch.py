"""Frame batches (sift_hip_set_batch / sift_hip_detect_batch_device): every
launch of the pipeline processes B frames.  Each frame's results must be those
of the single-frame pipeline on the same frame, bit for bit -- keypoints,
features AND descriptors (the fixed-point descriptor histogram is order
independent, so even the +-1 descriptor tolerance against the oracle does not
apply between the two GPU paths).  Covers full batches (graph), partial
batches (eager launches), 8-bit frames, upscale (firstOctave -1), a
single-frame call on a batch handle, and one frame against the CPU oracle.
"""
import numpy as np
import pytest
import torch
from parity_bar import assert_descriptor_bar


pytestmark = pytest.mark.gpu


def single_results(sift, cfg, frames, exact=False):
    det = sift.Detector(cfg, device=0, exact_descriptors=exact)
    det.gpuWarmUpAndAllocate()
    out = []
    for f in frames:
        det.detectAndCompute(f)
        det.copyToHost(True)
        out.append((det.final_kpts.copy(), det.final_features.copy(), det.descriptors.view(np.uint16).copy()))
    return out


def batch_results(sift, cfg, frames, B, u8=False, exact=False):
    det = sift.Detector(cfg, device=0, batch=B, exact_descriptors=exact)
    det.gpuWarmUpAndAllocate()
    dt = torch.uint8 if u8 else torch.float32
    t = torch.from_numpy(np.stack(frames)).to(dtype=dt, device="cuda:0").contiguous()
    h, w = frames[0].shape
    es = 1 if u8 else 4
    det.detectBatchDevice(t.data_ptr(), len(frames), w * es, h * w * es, u8=u8)
    assert det.batch_frames() == len(frames)
    out = []
    for i in range(len(frames)):
        n, ovf, *_ = det.batch_results(i)
        assert ovf == 0
        k3, f4, d = det.batch_copy_to_host(i)
        assert len(k3) == n
        out.append((k3, f4, d.view(np.uint16)))
    return det, out


def assert_equal_results(a, b):
    assert len(a) == len(b)
    for (k1, f1, d1), (k2, f2, d2) in zip(a, b):
        assert len(k1) > 20
        assert np.array_equal(k1, k2) and np.array_equal(f1, f2) and np.array_equal(d1, d2)


@pytest.mark.parametrize("B,n", [(3, 3), (4, 2)])
def test_batch_equals_single_frames(sift, B, n):
    w, h = 640, 360
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=1500, numOctaves=0)
    frames = [sift.synth_frame(40 + i, w, h) for i in range(n)]
    _, got = batch_results(sift, cfg, frames, B)
    assert_equal_results(got, single_results(sift, cfg, frames))


def test_batch_c2_workload_u8(sift):
    """The bench workload (1920x1200, 3 octaves, numFeatures 5000) as 8-bit frames."""
    w, h = 1920, 1200
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=5000, numOctaves=3)
    frames = [sift.synth_frame(50 + i, w, h) for i in range(4)]
    _, got = batch_results(sift, cfg, [f.astype(np.uint8) for f in frames], 4, u8=True)
    assert_equal_results(got, single_results(sift, cfg, frames))


@pytest.mark.parametrize("B,n", [(16, 16), (16, 5)])
def test_batch_c2_workload_16(sift, B, n):
    """bench.py's default launch group: 16 frames of the C2 workload per launch
    (4-wave blur tiles, batch-sized keypoint grids), a full and a partial batch."""
    w, h = 1920, 1200
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=5000, numOctaves=3)
    frames = [sift.synth_frame(80 + i, w, h) for i in range(n)]
    _, got = batch_results(sift, cfg, frames, B)
    assert_equal_results(got, single_results(sift, cfg, frames))


def test_batch_upscale(sift):
    w, h = 320, 240
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, upscale=True, numFeatures=0)
    frames = [sift.synth_frame(60 + i, w, h) for i in range(2)]
    _, got = batch_results(sift, cfg, frames, 2)
    assert_equal_results(got, single_results(sift, cfg, frames))


def test_single_frame_call_on_batch_handle(sift, oracle):
    w, h = 752, 480
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=0, numOctaves=3)
    frames = [sift.synth_frame(70 + i, w, h) for i in range(3)]
    det, got = batch_results(sift, cfg, frames, 3)
    det.detectAndCompute(frames[1])  # one-frame graph on the batch handle
    det.copyToHost(True)
    assert np.array_equal(det.final_kpts, got[1][0]) and np.array_equal(det.descriptors.view(np.uint16), got[1][2])
    # batch frame 2 against the CPU oracle (keypoints bit-exact, descriptors +-1)
    gk = np.stack([got[2][0][:, 0], got[2][0][:, 1], got[2][1][:, 1], got[2][1][:, 3], got[2][1][:, 2],
                   got[2][1][:, 0]], 1)
    ok, od = oracle.detect_and_compute(frames[2], oracle.from_config(cfg))
    assert len(ok) == len(gk) > 50
    o = np.stack([ok["x"], ok["y"], ok["size"], ok["angle"]], 1)
    gi, oi = np.lexsort(gk[:, :4].T[::-1]), np.lexsort(o.T[::-1])
    assert np.array_equal(gk[gi, :4], o[oi])
    assert_descriptor_bar(got[2][2].view(np.float16).astype(np.float32)[gi], od[oi], "batch frame 2")


def test_batch_exact_descriptors(sift, oracle):
    """SIFT_HIP_DESC_EXACT on a batch handle (full batch through the graph):
    frame results equal the single-frame exact handle's, and a frame's
    descriptors equal the oracle's byte for byte."""
    w, h = 752, 480
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=0, numOctaves=3)
    frames = [sift.synth_frame(90 + i, w, h) for i in range(4)]
    _, got = batch_results(sift, cfg, frames, 4, exact=True)
    assert_equal_results(got, single_results(sift, cfg, frames, exact=True))
    k3, f4, d = got[3]
    gk = np.stack([k3[:, 0], k3[:, 1], f4[:, 1], f4[:, 3], f4[:, 2]], 1)
    ok, od = oracle.detect_and_compute(frames[3], oracle.from_config(cfg))
    o = np.stack([ok["x"], ok["y"], ok["size"], ok["angle"], ok["response"]], 1)
    gi, oi = np.lexsort(gk.T[::-1]), np.lexsort(o.T[::-1])
    assert np.array_equal(gk[gi], o[oi])
    assert np.array_equal(d.view(np.float16).astype(np.float32)[gi], od[oi])

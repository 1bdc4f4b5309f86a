"""Frames in flight at the drop-in API ("Frames in flight").

A handle runs frames submitted before their predecessors complete on up to
`lanes` compute lanes (stream + frame arenas + graphs each).  Bar: every frame's
keypoints, features and descriptors -- and prev_descriptor -- are bit for bit
those of the synchronous one-frame-at-a-time path, whatever lane ran it; a
synchronous caller never creates a second lane; the in-flight limits hold.
Also (round-4 advisor): device frames from different buffers enqueued back to
back without a host sync, results copied out stream-ordered, equal the
synchronous results; device and host memory stay flat over a long loop.
"""
import ctypes

import numpy as np
import pytest
import torch

from test_gpu_input import assert_identical, results
from test_gpu_parity import make_detector

pytestmark = pytest.mark.gpu

W, H = 752, 480


def sync_reference(sift, frames, **kw):
    _, det = make_detector(sift, W, H, lanes=1, **kw)
    out = []
    for f in frames:
        det.detectAndCompute(f)
        out.append(results(det))
    assert det.lanes() == (1, 1)
    return out


def prev_rows(sift, det, n):
    prev = np.empty((n, 128), np.uint16)
    if n:
        sift._check(sift.lib().sift_hip_memcpy_d2h(prev.ctypes.data, det.prev_descriptor.data(), prev.nbytes), "d2h")
    return prev


def run_pipelined(sift, det, frames, ref, depth, submit, prev0=None):
    """Keeps `depth` frames in flight; each waited frame must equal the synchronous path
    (prev0: the reference of the frame before the first one, None for none)."""
    queue, i = [], 0

    def drain_one():
        nonlocal i
        t = queue.pop(0)
        det.wait(t)
        assert_identical(results(det), ref[i])
        before = ref[i - 1] if i else prev0
        if before is not None:
            assert det.prev_size == len(before[0])
            assert np.array_equal(prev_rows(sift, det, det.prev_size), before[2])
        else:
            assert det.prev_size == 0
        i += 1

    for s in range(len(frames)):
        queue.append(submit(s))
        if len(queue) == depth:
            drain_one()
    while queue:
        drain_one()
    assert i == len(frames)


@pytest.mark.parametrize("lanes,depth", [(2, 2), (3, 3), (4, 4), (2, 4)])
def test_host_submit_lanes_equal_sync(sift, lanes, depth):
    frames = [sift.synth_frame(50 + i, W, H) for i in range(10)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=lanes)
    run_pipelined(sift, det, frames, ref, depth,
                  lambda s: det.submit(frames[s].astype(np.uint8) if s % 3 == 1 else frames[s]))
    assert 1 <= det.lanes()[1] <= lanes


def test_device_submit_lanes_equal_sync(sift):
    frames = [sift.synth_frame(70 + i, W, H) for i in range(9)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    dev = [torch.from_numpy(f).cuda() for f in frames]
    u8 = [torch.from_numpy(f.astype(np.uint8)).cuda() for f in frames]
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=3)
    run_pipelined(sift, det, frames, ref, 3,
                  lambda s: det.submitDevice(u8[s].data_ptr(), W, u8=True) if s % 2
                  else det.submitDevice(dev[s].data_ptr(), W * 4))


@pytest.mark.parametrize("mb,lanes,depth", [(4, 2, 8), (4, 2, 3), (3, 3, 9), (2, 1, 4)])
def test_device_submit_micro_batch_equal_sync(sift, mb, lanes, depth):
    """Micro-batching (sift_hip_set_micro_batch): frames queue into launch
    groups of mb; full groups, partial groups launched by a wait on a queued
    frame (depth < mb), format changes inside a group, and frames ordered after
    the caller's stream all give the synchronous path's results and
    prev_descriptor."""
    frames = [sift.synth_frame(110 + i, W, H) for i in range(13)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    dev = [torch.from_numpy(f).cuda() for f in frames]
    u8 = [torch.from_numpy(f.astype(np.uint8)).cuda() for f in frames]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=lanes, micro_batch=mb)
    assert det.micro_batch() == mb

    def submit(s):
        if s % 5 == 3:  # a u8 frame inside a group of f32 frames: converted, the group runs as f32
            return det.submitDevice(u8[s].data_ptr(), W, u8=True)
        if s % 4 == 1:
            return det.submitDevice(dev[s].data_ptr(), W * 4, stream=stream.cuda_stream)
        return det.submitDevice(dev[s].data_ptr(), W * 4)

    run_pipelined(sift, det, frames, ref, depth, submit)
    # a synchronous detect between queued frames launches them first, in order
    t0 = det.submitDevice(dev[0].data_ptr(), W * 4)
    det.detectAndComputeDevice(dev[1].data_ptr(), W * 4, sync=True)
    assert_identical(results(det), ref[1])
    det.wait(t0)
    assert_identical(results(det), ref[0])


def test_batch_accessors_on_micro_batch_frames(sift):
    """(Round-5 advisor.)  A waited frame of a micro-batch has its own frame
    number: the batch accessors expose that frame alone (batch_frames 1, index
    0 = the frame's own results and counters, index 1 refused), never arenas
    past the frame's group -- whichever arena of the group it ran in."""
    frames = [sift.synth_frame(140 + i, W, H) for i in range(8)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    dev = [torch.from_numpy(f).cuda() for f in frames]
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=2, micro_batch=4)
    tickets = [det.submitDevice(d.data_ptr(), W * 4) for d in dev]
    for i, t in enumerate(tickets):
        det.wait(t)
        assert det.batch_frames() == 1
        n, ovf, k3p, f4p, dp = det.batch_results(0)
        assert n == det.total_size == len(ref[i][0]) and ovf == det.overflow_flags()
        assert dp == det.device_descriptor.data()
        k3, f4, d = det.batch_copy_to_host(0)
        assert np.array_equal(k3, ref[i][0]) and np.array_equal(d.view(np.uint16), ref[i][2])
        with pytest.raises(RuntimeError):
            det.batch_results(1)


@pytest.mark.parametrize("mb,lanes,depth", [(4, 2, 8), (3, 3, 2)])
def test_host_submit_micro_batch_equal_sync(sift, mb, lanes, depth):
    """Host frames on a micro-batching handle: staged into the handle's pinned
    ring, copied into the group input by the group's lane, results prefetched
    per frame to pinned host memory (copyToHost after every wait); host and
    device frames share groups."""
    frames = [sift.synth_frame(130 + i, W, H) for i in range(11)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    dev = [torch.from_numpy(f).cuda() for f in frames]
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=lanes, micro_batch=mb)

    def submit(s):
        if s % 4 == 2:
            return det.submitDevice(dev[s].data_ptr(), W * 4)
        return det.submit(frames[s].astype(np.uint8) if s % 3 == 1 else frames[s])

    run_pipelined(sift, det, frames, ref, depth, submit)
    det.detectAndCompute(frames[5])  # a synchronous host frame: a group of one
    assert_identical(results(det), ref[5])


def view_results(det):
    k3, f4, d = det.results_host(True)
    return k3, f4, d.view(np.uint16)


@pytest.mark.parametrize("mb,lanes,depth", [(1, 3, 6), (4, 3, 12), (3, 2, 4), (8, 3, 24)])
def test_results_host_views_equal_sync(sift, mb, lanes, depth):
    """sift_hip_results_host: the current frame's rows as views of the handle's
    pinned results (no copy into caller memory) equal the synchronous path's
    for host frames (written there by the frame's last kernel) and device
    frames (copied there by the call), and a frame's views stay intact while
    it is the previous frame (the next frame waited, later frames in flight)."""
    frames = [sift.synth_frame(150 + i, W, H) for i in range(12)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    dev = [torch.from_numpy(f).cuda() for f in frames]
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=lanes, micro_batch=mb)
    queue, i, prev = [], 0, None

    def drain_one():
        nonlocal i, prev
        det.wait(queue.pop(0))
        if i % 5 == 4:  # keypoints only first: the descriptor rows come on the next request
            k3, f4, d = det.results_host(False)
            assert d is None
            assert_identical((k3, f4), ref[i][:2])
        cur = view_results(det)
        assert_identical(cur, ref[i])
        if prev is not None:
            assert_identical(prev, ref[i - 1])
        prev = cur
        i += 1

    for s in range(len(frames)):
        queue.append(det.submitDevice(dev[s].data_ptr(), W * 4) if s % 3 == 2
                     else det.submit(frames[s].astype(np.uint8) if s % 2 else frames[s]))
        if len(queue) == depth:
            drain_one()
    while queue:
        drain_one()
    det.detectAndCompute(frames[3])  # synchronous: copied by the call
    assert_identical(view_results(det), ref[3])
    _, det0 = make_detector(sift, W, H, numFeatures=2000)
    det0.detectAndCompute(frames[0])
    assert_identical(view_results(det0), ref[0])  # first call on a handle (regions allocated by it)


@pytest.mark.parametrize("kw,mb", [({"upscale": True}, 2), ({"exact_descriptors": True}, 3),
                                   ({"upscale": True, "exact_descriptors": True}, 1)])
def test_host_rows_other_heads_and_exact_kernel(sift, kw, mb):
    """The host rows written by the descriptor kernel (HostOut) on the other
    paths that carry the request: a doubled base (the request crosses the
    upsample head and survives the body's first blur) and the exact
    descriptor kernel; results_host and copyToHost both equal the sync path."""
    w, h = 320, 240
    frames = [sift.synth_frame(170 + i, w, h) for i in range(7)]
    _, ref_det = make_detector(sift, w, h, numFeatures=1500, lanes=1, **kw)
    ref = []
    for f in frames:
        ref_det.detectAndCompute(f)
        ref.append(results(ref_det))
    _, det = make_detector(sift, w, h, numFeatures=1500, lanes=2, micro_batch=mb, **kw)
    queue, i = [], 0
    for s in range(len(frames)):
        queue.append(det.submit(frames[s].astype(np.uint8) if s % 2 else frames[s]))
        if len(queue) == 3:
            det.wait(queue.pop(0))
            assert_identical(view_results(det) if i % 2 else results(det), ref[i])
            i += 1
    while queue:
        det.wait(queue.pop(0))
        assert_identical(view_results(det), ref[i])
        i += 1


def test_micro_batch_limits(sift):
    img = torch.from_numpy(sift.synth_frame(1, 128, 96)).cuda()
    torch.cuda.synchronize()
    _, det = make_detector(sift, 128, 96, lanes=1, micro_batch=2)
    t = [det.submitDevice(img.data_ptr(), 128 * 4) for _ in range(4)]  # two groups of 2 on the one lane
    with pytest.raises(sift.SiftHipError):
        det.submitDevice(img.data_ptr(), 128 * 4)
    for x in t:
        det.wait(x)
    with pytest.raises(sift.SiftHipError):
        sift.Detector(sift.CudaSiftConfig(col_width=128, row_width=96), micro_batch=17)
    with pytest.raises(sift.SiftHipError):  # batch and micro-batch must agree
        d2 = sift.Detector(sift.CudaSiftConfig(col_width=128, row_width=96), batch=4, micro_batch=2)
        d2.gpuWarmUpAndAllocate()


def test_sync_caller_keeps_one_lane(sift):
    _, det = make_detector(sift, W, H, numFeatures=2000)
    img = sift.synth_frame(3, W, H)
    for _ in range(4):
        det.detectAndCompute(img)
    dev = torch.from_numpy(img).cuda()
    torch.cuda.synchronize()
    for _ in range(3):
        det.detectAndComputeDevice(dev.data_ptr(), W * 4, sync=True)
    assert det.lanes() == (2, 1)


def test_lane_limits(sift):
    img = sift.synth_frame(1, 128, 96)
    _, det = make_detector(sift, 128, 96, lanes=2, auto_micro_batch=0)  # unbatched: 2 frames per lane
    assert det.auto_micro_batch() == 0
    t = [det.submit(img) for _ in range(4)]  # two per lane past the current frame
    with pytest.raises(sift.SiftHipError):
        det.submit(img)
    det.wait(t[1])
    det.wait(t[0])  # frames current-1 .. on stay readable
    t.append(det.submit(img))
    for x in t[2:]:
        det.wait(x)
    with pytest.raises(sift.SiftHipError):
        sift.Detector(sift.CudaSiftConfig(col_width=128, row_width=96), lanes=5)


@pytest.mark.parametrize("lanes,depth,n", [(3, 12, 26), (3, 24, 40), (2, 12, 30), (4, 36, 50)])
def test_device_submit_auto_groups_equal_sync(sift, lanes, depth, n):
    """Automatic launch groups (the default: sift_hip_set_auto_micro_batch 8):
    a caller keeping `depth` device frames in flight with no micro-batch call
    gets its frames queued once every lane is busy and run in groups of up to
    8 on the lanes created after lane 0; every waited frame and
    prev_descriptor equal the synchronous path, u8 frames and frames ordered
    after the caller's stream included."""
    frames = [sift.synth_frame(300 + i % 13, W, H) for i in range(n)]
    ref13 = sync_reference(sift, frames[:13], numFeatures=2000)
    ref = [ref13[i % 13] for i in range(n)]
    dev = [torch.from_numpy(f).cuda() for f in frames[:13]]
    u8 = [torch.from_numpy(f.astype(np.uint8)).cuda() for f in frames[:13]]
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=lanes)
    assert det.auto_micro_batch() == 8 and det.micro_batch() == 1

    def submit(s):
        if s % 7 == 5:
            return det.submitDevice(u8[s % 13].data_ptr(), W, u8=True)
        if s % 4 == 1:
            return det.submitDevice(dev[s % 13].data_ptr(), W * 4, stream=stream.cuda_stream)
        return det.submitDevice(dev[s % 13].data_ptr(), W * 4)

    # frame i's reference predecessor is frame i - 1 of the same sequence (ref[i - 1])
    run_pipelined(sift, det, frames, ref, depth, submit)
    assert det.lanes()[1] >= 2
    # the in-flight limit, max(2 x lanes, (lanes - 1) x 3 x 4) frames past the current one, and not
    # a submit earlier (every frame up to it finds a results slot)
    limit, ok = max(2 * lanes, (lanes - 1) * 12), 0
    with pytest.raises(sift.SiftHipError, match="in flight"):
        for _ in range(limit + 1):
            det.submitDevice(dev[0].data_ptr(), W * 4)
            ok += 1
    assert ok == limit
    det.sync()
    # a synchronous detect after the stream: lane 0, one frame
    det.detectAndComputeDevice(dev[2].data_ptr(), W * 4, sync=True)
    assert_identical(results(det), ref13[2])


@pytest.mark.parametrize("depth", [6, 20, 24])
def test_host_submit_auto_groups_equal_sync(sift, depth):
    """Host frames (f32 and u8) under automatic launch groups: staged into the
    pinned ring once queued, results read back after every wait.  Three passes
    on one handle: each restarts from a drained pipeline (single frames, then
    groups), the transition that once left group lanes' results slots holding
    single frames still readable (round 6: 8 slots on those lanes)."""
    frames = [sift.synth_frame(330 + i, W, H) for i in range(30)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    _, det = make_detector(sift, W, H, numFeatures=2000, lanes=3)
    for p in range(3):
        run_pipelined(sift, det, frames, ref, depth,
                      lambda s: det.submit(frames[s].astype(np.uint8) if s % 3 == 1 else frames[s]),
                      prev0=ref[-1] if p else None)


class _Cai:
    """A raw device pointer as a torch tensor (__cuda_array_interface__), no copy."""

    def __init__(self, ptr, shape, typestr):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (ptr, False), "version": 2}


def test_device_frames_back_to_back_stream_ordered(sift):
    """Round-4 advisor: >= 5 device frames from different buffers enqueued
    without a host sync (the frame graph's head node re-pointed per frame, or
    the separate head launch while that graph is still in flight); each
    frame's results copied out on the caller's stream right after it."""
    frames = [sift.synth_frame(90 + i, W, H) for i in range(8)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    bufs = [torch.from_numpy(f).cuda() for f in frames]
    # a real stream: torch's default one is the null stream (no handle to order on)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000)
    cap = det.capacities()["results"]
    lib = sift.lib()
    outs = []
    ctx = torch.cuda.stream(stream)
    ctx.__enter__()
    for b in bufs:
        det.detectAndComputeDevice(b.data_ptr(), W * 4, stream=stream.cuda_stream, sync=False)
        k3, f4, d = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        sift._check(lib.sift_hip_results_device(det.handle, ctypes.byref(k3), ctypes.byref(f4), ctypes.byref(d),
                                                None, None, None), "results_device")
        outs.append((torch.as_tensor(_Cai(k3.value, (cap, 3), "<f4"), device="cuda").clone(),
                     torch.as_tensor(_Cai(f4.value, (cap, 4), "<f4"), device="cuda").clone(),
                     torch.as_tensor(_Cai(d.value, (cap, 128), "<i2"), device="cuda").clone()))
    ctx.__exit__(None, None, None)
    torch.cuda.synchronize()
    det.sync()
    assert det.total_size == len(ref[-1][0])
    for (k, f, d), r in zip(outs, ref):
        n = len(r[0])
        got = (k[:n].cpu().numpy(), f[:n].cpu().numpy(), d[:n].cpu().numpy().view(np.uint16))
        assert_identical(got, r)


def test_long_loop_memory_flat(sift):
    import os

    import psutil

    frames = [torch.from_numpy(sift.synth_frame(i, W, H)).cuda() for i in range(4)]
    torch.cuda.synchronize()
    _, det = make_detector(sift, W, H, numFeatures=2000)
    proc = psutil.Process(os.getpid())

    def run(n):
        for s in range(n):
            det.detectAndComputeDevice(frames[s % 4].data_ptr(), W * 4, sync=(s % 10 == 9))
        det.sync()

    run(50)  # both lanes created, graphs warm
    free0, rss0 = torch.cuda.mem_get_info()[0], proc.memory_info().rss
    run(400)
    free1, rss1 = torch.cuda.mem_get_info()[0], proc.memory_info().rss
    assert abs(free1 - free0) <= 4 << 20, f"device memory moved by {(free0 - free1) / 2**20:.1f} MiB"
    assert rss1 - rss0 <= 32 << 20, f"host RSS grew by {(rss1 - rss0) / 2**20:.1f} MiB"


@pytest.mark.parametrize("u8", [False, True])
def test_strided_large_host_frames(sift, u8):
    """Host frames of >= 1 MB are staged by the copy pool (row ranges split over
    threads): contiguous and strided (a view into a wider buffer) frames give
    the results of the same frame through the device path."""
    w, h = 1920, 1200
    img = sift.synth_frame(4, w, h)
    src = img.astype(np.uint8) if u8 else img
    _, det = make_detector(sift, w, h, numOctaves=3, lanes=1)
    dev = torch.from_numpy(img).cuda()
    torch.cuda.synchronize()
    det.detectAndComputeDevice(dev.data_ptr(), w * 4, sync=True)
    ref = results(det)
    det.detectAndCompute(src)
    assert_identical(results(det), ref)
    wide = np.zeros((h, w + 29), src.dtype)
    wide[:, 3:3 + w] = src
    det.detectAndCompute(wide[:, 3:3 + w])
    assert_identical(results(det), ref)
    det.copyToHost(False)  # keypoints only, from the same host copy
    assert np.array_equal(det.final_kpts.view(np.uint32), ref[0].view(np.uint32))


def test_host_frames_on_large_batch_handle(sift):
    """A 32-frame batch handle taking host frames with results read back
    (per-(slot, arena) host regions up to slot 3 x 32): the synchronous path's results."""
    frames = [sift.synth_frame(150 + i, W, H) for i in range(6)]
    ref = sync_reference(sift, frames, numFeatures=2000)
    det = sift.Detector(sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=2000), batch=32, lanes=1)
    det.gpuWarmUpAndAllocate()
    for f, r in zip(frames, ref):
        det.detectAndCompute(f)
        assert_identical(results(det), r)
    q = [det.submit(f) for f in frames[:2]]
    for t, r in zip(q, ref[:2]):
        det.wait(t)
        assert_identical(results(det), r)

"""Stage dumps (Detector::setDataGen): a detect with
dumps on writes every stage of the frame, and the replay (tests/stage_check.py)
finds the dump consistent with the CPU oracle stage by stage and with a fresh
detector run on the dumped input, bit for bit."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import stage_check

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("w,h,upscale,u8", [(400, 300, False, False), (257, 191, True, True)])
def test_datagen_dump_replays(sift, tmp_path, w, h, upscale, u8):
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, upscale=upscale, numFeatures=0)
    det = sift.Detector(cfg, device=0)
    det.gpuWarmUpAndAllocate()
    out = str(tmp_path / "dump")
    det.setDataGen(out)
    img = sift.synth_frame(12, w, h)
    det.detectAndCompute(img.astype(np.uint8) if u8 else img)
    det.copyToHost(True)
    d = stage_check.load(out)
    assert d["meta"]["keypoints"] == det.total_size > 20
    assert np.array_equal(d["input"], img)
    assert np.array_equal(d["desc"].view(np.uint16), det.descriptors.view(np.uint16))
    res = stage_check.check_oracle(d)
    assert all(v for v in res.values() if isinstance(v, bool)), res
    rep = stage_check.check_gpu(d)
    assert all(rep.values()), rep
    # switched off: the next frame leaves the dump alone
    det.setDataGen("")
    det.detectAndCompute(sift.synth_frame(13, w, h))
    assert stage_check.load(out)["meta"]["keypoints"] == d["meta"]["keypoints"]


def test_stage_check_cli(sift, tmp_path):
    w, h = 320, 240
    det = sift.Detector(sift.CudaSiftConfig(col_width=w, row_width=h), device=0)
    det.gpuWarmUpAndAllocate()
    det.setDataGen(str(tmp_path))
    det.detectAndCompute(sift.synth_frame(3, w, h))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "stage_check.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout)["oracle"]["keypoints_bitexact"]


@pytest.mark.parametrize("w,h,upscale,exact", [(400, 300, False, False), (257, 191, True, False),
                                              (400, 300, False, True)])
def test_stage_replay_each_stage(sift, tmp_path, w, h, upscale, exact):
    """Per-stage replay (tool/perf.cu:43-100): every stage's kernels alone on
    the dump's recorded input reproduce the dump's output of that stage bit for
    bit (as record sets where the device appends with atomics); the handle then
    detects normally again.  Also with the exact descriptor mode (the replayed
    descriptor stage is the exact kernel)."""
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, upscale=upscale, numFeatures=0)
    det = sift.Detector(cfg, device=0, exact_descriptors=exact)
    det.gpuWarmUpAndAllocate()
    dump = str(tmp_path / "dump")
    det.setDataGen(dump)
    img = sift.synth_frame(14, w, h)
    det.detectAndCompute(img)
    det.setDataGen("")
    want_n = det.total_size
    d = stage_check.load(dump)
    assert d["meta"]["format"] == "sift_hip stage dump 2" and want_n > 20
    res = stage_check.check_stages(dump, det=det, out_root=str(tmp_path / "replay"))
    assert res == {s: True for s in stage_check.STAGES}, res
    # after a replay the handle is as after warm-up: the next frame is normal
    det.detectAndCompute(img)
    det.copyToHost(True)
    assert det.total_size == want_n and np.array_equal(det.descriptors.view(np.uint16), d["desc"].view(np.uint16))


def test_stage_replay_uses_the_dumped_input(sift, tmp_path):
    """The descriptor stage reads the dump's jobs: one job's angle changed by
    90 degrees changes that keypoint's descriptor only; one refined record
    moved by a pixel changes only what the orientation stage emits for it."""
    w, h = 320, 240
    det = sift.Detector(sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=0), device=0)
    det.gpuWarmUpAndAllocate()
    dump = str(tmp_path / "dump")
    det.setDataGen(dump)
    det.detectAndCompute(sift.synth_frame(15, w, h))
    det.setDataGen("")
    jobs = np.fromfile(os.path.join(dump, "jobs.rec"), np.uint32).reshape(-1, 16)
    ang = jobs[:, 4].view(np.float32)  # {i64 plane, f32 cos_t, sin_t, angle, ...}
    ang[3] = (ang[3] + 90.0) % 360.0
    cs = jobs[:, 2:4].view(np.float32)
    cs[3] = np.array([-cs[3, 1], cs[3, 0]], np.float32)  # rotate (cos, sin) with it
    jobs.tofile(os.path.join(dump, "jobs.rec"))
    out = str(tmp_path / "desc")
    det.replayStage(dump, "descriptor", out)
    got = np.fromfile(os.path.join(out, "desc.f16"), np.uint16).reshape(-1, 128)
    ref = np.fromfile(os.path.join(dump, "desc.f16"), np.uint16).reshape(-1, 128)
    rows = np.nonzero(np.any(got != ref, 1))[0]
    assert list(rows) == [int(jobs[3, 12])]  # the job's output row (DescJob.out)
    with pytest.raises(sift.SiftHipError):
        det.replayStage(dump, "no-such-stage", out)


@pytest.mark.parametrize("stage", ["descriptor", "refine", "pyramid"])
def test_stage_replay_failed_write_restores_handle(sift, tmp_path, stage):
    """A replay whose output write fails after its kernels ran (the output file
    name is taken by a directory) reports the error and still leaves the
    handle as after warm-up: timing mode restored, the arena's
    scratch invariants (counters, dedupe bitmap, range keys) reset, so the next
    frame is bit-exact with the one before the replay."""
    w, h = 320, 240
    det = sift.Detector(sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=0), device=0)
    det.gpuWarmUpAndAllocate()
    dump = str(tmp_path / "dump")
    img = sift.synth_frame(16, w, h)
    det.setDataGen(dump)
    det.detectAndCompute(img)
    det.setDataGen("")
    det.copyToHost(True)
    want_k, want_d = det.final_kpts.copy(), det.descriptors.view(np.uint16).copy()
    out = tmp_path / "out"
    blocker = {"descriptor": "desc.f16", "refine": "refined.rec", "pyramid": "gauss_o0_l0.f32"}[stage]
    os.makedirs(out / blocker)  # fopen(out/blocker, "wb") fails after the stage's kernels
    det.set_timing(True)
    with pytest.raises(sift.SiftHipError):
        det.replayStage(dump, stage, str(out))
    det.timing_reset()
    det.detectAndCompute(img)  # timing mode still on: the stages record their launches
    assert det.timing().get("descriptor", {}).get("launches", 0) == 1
    det.copyToHost(True)
    assert np.array_equal(det.final_kpts, want_k)
    assert np.array_equal(det.descriptors.view(np.uint16), want_d)
    det.set_timing(False)
    det.detectAndCompute(img)
    det.copyToHost(True)
    assert np.array_equal(det.descriptors.view(np.uint16), want_d)

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

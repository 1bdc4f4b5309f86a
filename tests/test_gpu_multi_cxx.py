"""The C++ multi-GPU caller on the GPU (tools/multi_gpu_example.cpp over
sift_cuda::MultiDetector / crossMatch): two workers (detectors on their own
host threads; on a one-GPU box both on GPU 0) shard the frames, every frame's
keypoint count equals a single Python detector's, and the cross match of the
two workers' descriptor sets equals the Python matcher's on the same sets."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "another-cuda-sift_amd", "lib", "multi_gpu_example")


def test_multi_gpu_example_virtual(sift):
    w, h, frames, rows = 640, 360, 8, 500
    r = subprocess.run([EXE, "--virtual", "2", "--frames", str(frames), "--width", str(w), "--height", str(h),
                        "--rows", str(rows)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["workers"] == 2 and out["frames"] == frames and out["gather"] == "copy"
    cfg = sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=5000)
    det = sift.Detector(cfg, device=0)
    det.gpuWarmUpAndAllocate()
    descs = []
    for f in range(frames):
        det.detectAndCompute(sift.synth_frame(f, w, h).astype(np.uint8))
        assert out["kpts"][f] == det.total_size, f
        if f < 2:
            det.copyToHost(True)
            descs.append(det.descriptors[:rows].copy())
    dev = []
    for d in descs:
        pad = np.zeros((rows, 128), np.float16)
        pad[:len(d)] = d
        dev.append(sift.DeviceArray.from_numpy(pad))
    m = sift.Matcher(rows, rows)
    want = {}
    for k, j in ((0, 1), (1, 0)):
        mt = sift.DeviceArray(rows * 4)
        m.match_device(dev[k].value, len(descs[k]), dev[j].value, len(descs[j]), 0.8, False, 0, 0, mt.value)
        want[(k, j)] = int((mt.to_numpy(np.int32, (rows,))[:len(descs[k])] >= 0).sum())
    got = {(k, j): g for k, j, g in out["matches"]}
    assert got == want
    assert out["set_rows"] == [len(d) for d in descs]

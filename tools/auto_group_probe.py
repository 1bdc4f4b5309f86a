"""Frames in flight on a default handle (automatic launch groups) against an
explicit micro-batch: host u8 frames with every frame's results copied back,
and device f32 frames, submit/wait at a fixed depth, rounds interleaved.
Usage (GPU box): SIFT_HIP_LIB=ab/X.so python tools/auto_group_probe.py TAG"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "another-cuda-sift_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sift_amd as sift  # noqa: E402

W, H, N, DEPTH = 1920, 1200, 192, 24
tag = sys.argv[1] if len(sys.argv) > 1 else "run"
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=3)
host8 = [sift.synth_frame(i, W, H).astype(np.uint8) for i in range(4)]
dev = [torch.from_numpy(sift.synth_frame(i, W, H)).cuda() for i in range(4)]
torch.cuda.synchronize()


def loop(det, submit, fetch):
    q = []
    for s in range(N + 2 * DEPTH):
        if s == 2 * DEPTH:
            while q:
                det.wait(q.pop(0))
                if fetch:
                    det.copyToHost(True)
            t = time.perf_counter()
        q.append(submit(s))
        if len(q) == DEPTH:
            det.wait(q.pop(0))
            if fetch:
                det.copyToHost(True)
    while q:
        det.wait(q.pop(0))
        if fetch:
            det.copyToHost(True)
    return round((time.perf_counter() - t) / N * 1e3, 4)


auto = sift.Detector(cfg, lanes=3)
auto.gpuWarmUpAndAllocate()
mb = sift.Detector(cfg, lanes=3, micro_batch=8)
mb.gpuWarmUpAndAllocate()
for r in range(3):
    rec = {"tag": tag, "round": r}
    for name, det in (("auto", auto), ("mb8", mb)):
        rec[f"{name}_host_u8_ms"] = loop(det, lambda s: det.submit(host8[s % 4]), True)
        rec[f"{name}_dev_f32_ms"] = loop(det, lambda s: det.submitDevice(dev[s % 4].data_ptr(), W * 4), False)
    rec["auto_lanes"] = list(auto.lanes())
    print(json.dumps(rec), flush=True)

"""Host / device submit-wait loops on a default handle (3 lanes), for A/B of
the lane scheduling: python tools/auto_ab.py [DEPTH ...] -> one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "another-cuda-sift_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sift_amd as sift  # noqa: E402

W, H, N = 1920, 1200, 200
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=3)
host8 = [sift.synth_frame(i, W, H).astype(np.uint8) for i in range(4)]
dev = [torch.from_numpy(sift.synth_frame(i, W, H)).cuda() for i in range(4)]
torch.cuda.synchronize()


def loop(det, depth, submit, fetch):
    q = []
    for s in range(N + 3 * depth):
        if s == 3 * depth:
            while q:
                det.wait(q.pop(0))
            t = time.perf_counter()
        q.append(submit(s))
        if len(q) == depth:
            det.wait(q.pop(0))
            if fetch:
                det.copyToHost(True)
    while q:
        det.wait(q.pop(0))
        if fetch:
            det.copyToHost(True)
    return (time.perf_counter() - t) / N * 1e3


out = {"lib": os.environ.get("SIFT_HIP_LIB", "default")}
det = sift.Detector(cfg, lanes=3)
det.gpuWarmUpAndAllocate()
for depth in [int(x) for x in sys.argv[1:]] or [6]:
    out[f"host_u8_d{depth}"] = round(loop(det, depth, lambda s: det.submit(host8[s % 4]), True), 4)
    out[f"dev_f32_d{depth}"] = round(loop(det, depth, lambda s: det.submitDevice(dev[s % 4].data_ptr(), W * 4), False), 4)
print(json.dumps(out), flush=True)

"""Device-input submit/wait throughput (C2 frames, HBM-resident, 8-bit and
f32) at lanes x depth, plus synchronous single-frame latency, for A/B builds
(SIFT_HIP_LIB).  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sift_amd as sift  # noqa: E402

W, H, N = 1920, 1200, 150
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=3)
dev = [torch.from_numpy(sift.synth_frame(i, W, H)).cuda() for i in range(4)]
torch.cuda.synchronize()
out = {"lib": os.environ.get("SIFT_HIP_LIB", "default"), "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "")}
# (lanes, depth, micro-batch); DEV_CONFIGS="l:d:m,..." overrides
CONFIGS = [(3, 3, 1), (3, 6, 1), (2, 4, 1), (4, 8, 1)]
if os.environ.get("DEV_CONFIGS"):
    CONFIGS = [tuple(int(x) for x in c.split(":")) for c in os.environ["DEV_CONFIGS"].split(",")]
for lanes, depth, mb in CONFIGS:
    det = sift.Detector(cfg, lanes=lanes, micro_batch=mb)
    det.gpuWarmUpAndAllocate()
    q = []
    for s in range(N + 2 * depth):
        if s == 2 * depth:
            while q:
                det.wait(q.pop(0))
            t = time.perf_counter()
        q.append(det.submitDevice(dev[s % 4].data_ptr(), W * 4))
        if len(q) == depth:
            det.wait(q.pop(0))
    while q:
        det.wait(q.pop(0))
    out[f"l{lanes}d{depth}" + (f"m{mb}" if mb > 1 else "") + "_ms"] = round((time.perf_counter() - t) / N * 1e3, 4)
    if lanes == 3 and depth == 3 and mb == 1:
        lat = []
        for s in range(40):
            t = time.perf_counter()
            det.detectAndComputeDevice(dev[s % 4].data_ptr(), W * 4, sync=True)
            lat.append(time.perf_counter() - t)
        out["sync_ms"] = round(float(np.median(lat)) * 1e3, 4)
    del det
print(json.dumps(out), flush=True)

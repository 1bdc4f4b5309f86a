"""C2 throughput (1920x1200, 3 octaves, numFeatures 5000, HBM-resident frames)
for combinations of frames per launch (--batches) and detectors/streams
(--streams): picks bench.py's defaults.  One JSON line per combination."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import torch  # noqa: E402  (HIP runtime first)
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", default="1,2,4,8")
ap.add_argument("--streams", default="1,2,3")
ap.add_argument("--frames", type=int, default=400, help="frames timed per combination")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1200)
ap.add_argument("--octaves", type=int, default=3)
ap.add_argument("--exact", action="store_true", help="exact descriptor mode (SIFT_HIP_DESC_EXACT)")
ap.add_argument("--lanes", type=int, default=0, help="lanes per detector (0: the handle default; bench.py uses 1)")
a = ap.parse_args()
W, H = a.width, a.height
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=a.octaves)
for B in [int(x) for x in a.batches.split(",")]:
    fb = torch.from_numpy(np.stack([sift.synth_frame(i, W, H) for i in range(B)])).cuda()
    for S in [int(x) for x in a.streams.split(",")]:
        kw = {"lanes": a.lanes} if a.lanes else {}
        dets = [sift.Detector(cfg, device=0, batch=B, exact_descriptors=a.exact, **kw) for _ in range(S)]
        for d in dets:
            d.gpuWarmUpAndAllocate()

        def step(k):
            d = dets[k % S]
            if B == 1:
                d.detectAndComputeDevice(fb.data_ptr(), W * 4, sync=False)
            else:
                d.detectBatchDevice(fb.data_ptr(), B, W * 4, W * H * 4, sync=False)

        for k in range(3 * S):
            step(k)
        for d in dets:
            d.sync()
        n = max(a.frames // B, 2 * S)
        t = time.perf_counter()
        for k in range(n):
            step(k)
        for d in dets:
            d.sync()
        dt = time.perf_counter() - t
        print(json.dumps({"batch": B, "streams": S, "ms_per_frame": round(dt / (n * B) * 1e3, 4),
                          "mpix_s": round(n * B * W * H / 1e6 / dt, 1), "kpts_frame0": dets[0].total_size}), flush=True)
        del dets

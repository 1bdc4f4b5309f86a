"""Synchronous single-frame latency at the reference's published
configurations (as bench.py run_ref_configs) and C2, for A/B builds:

    SIFT_HIP_LIB=ab/X.so python tools/lat_configs.py [--reps 40]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=40)
a = ap.parse_args()
out = {"lib": os.environ.get("SIFT_HIP_LIB", "default")}
for (w, h, noct) in ((752, 480, 0), (1920, 1200, 0), (1600, 900, 0), (1920, 1200, 3)):
    d = sift.Detector(sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=5000, upscale=False, numOctaves=noct),
                      device=0)
    d.gpuWarmUpAndAllocate()
    img = sift.DeviceArray.from_numpy(sift.synth_frame(0, w, h))
    for _ in range(5):
        d.detectAndComputeDevice(img.value, w * 4, sync=True)
    lat = []
    for _ in range(a.reps):
        t = time.perf_counter()
        d.detectAndComputeDevice(img.value, w * 4, sync=True)
        lat.append(time.perf_counter() - t)
    out[f"{w}x{h}x{noct or 'auto'}"] = {"sync_ms": round(float(np.median(lat)) * 1e3, 4), "octaves": d.nOctaves,
                                        "keypoints": d.total_size}
    del d, img
print(json.dumps(out))

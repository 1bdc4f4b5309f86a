"""C2 throughput and single-frame latency with the default (fixed-point) and
the exact (OpenCV sequential float) descriptor histogram.

    python3 tools/desc_mode_bench.py [--steps 30]

Same workload as bench.py (1920x1200, 3 octaves, numFeatures 5000, 16-frame
launches on two streams; single frames serialised on one handle); prints one
JSON line per mode."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import sift_amd as sift  # noqa: E402

W, H = 1920, 1200


def run(exact, steps, B=16, streams=2):
    cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=3)
    dets = [sift.Detector(cfg, device=0, batch=B, exact_descriptors=exact) for _ in range(streams)]
    for d in dets:
        d.gpuWarmUpAndAllocate()
    fb = torch.from_numpy(np.stack([sift.synth_frame(i, W, H) for i in range(B)])).cuda()
    for s in range(2 * streams):
        dets[s % streams].detectBatchDevice(fb.data_ptr(), B, W * 4, W * H * 4, sync=False)
    for d in dets:
        d.sync()
    t = time.perf_counter()
    for s in range(steps):
        dets[s % streams].detectBatchDevice(fb.data_ptr(), B, W * 4, W * H * 4, sync=False)
    for d in dets:
        d.sync()
    el = time.perf_counter() - t
    del dets
    det = sift.Detector(cfg, device=0, exact_descriptors=exact)
    det.gpuWarmUpAndAllocate()
    f1 = fb[0].contiguous()
    lat = []
    for _ in range(20):
        t = time.perf_counter()
        det.detectAndComputeDevice(f1.data_ptr(), W * 4, sync=True)
        lat.append(time.perf_counter() - t)
    return {"mode": "exact" if exact else "fast", "mpix_per_s": round(steps * B * W * H / 1e6 / el, 1),
            "ms_per_frame": round(el / (steps * B) * 1e3, 4), "single_sync_ms_median": round(float(np.median(lat)) * 1e3, 4),
            "keypoints_frame0": det.total_size}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    for exact in (False, True):
        print(json.dumps(run(exact, a.steps)), flush=True)


if __name__ == "__main__":
    main()

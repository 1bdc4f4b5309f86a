"""Frames in flight at the drop-in API: submit/wait throughput by lanes and
depth (device and host input), and the host path's per-call costs.
Usage (GPU box): python tools/lanes_probe.py > gpurun_out/lanes_probe.jsonl"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "another-cuda-sift_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sift_amd as sift  # noqa: E402

W, H, N = 1920, 1200, 120
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, numOctaves=3)
host = [sift.synth_frame(i, W, H) for i in range(4)]
host8 = [f.astype(np.uint8) for f in host]
dev = [torch.from_numpy(f).cuda() for f in host]
dev8 = [torch.from_numpy(f).cuda() for f in host8]
torch.cuda.synchronize()


def loop(det, depth, submit, fetch=False, n=N):
    q = []
    for s in range(n + depth):
        if s == depth:
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
    return (time.perf_counter() - t) / n * 1e3


for lanes in (1, 2, 3, 4):
    det = sift.Detector(cfg, lanes=lanes)
    det.gpuWarmUpAndAllocate()
    for depth in sorted({lanes, 2 * lanes}):
        r = {"lanes": lanes, "depth": depth}
        r["device_f32_ms"] = round(loop(det, depth, lambda s: det.submitDevice(dev[s % 4].data_ptr(), W * 4)), 4)
        r["device_u8_ms"] = round(loop(det, depth, lambda s: det.submitDevice(dev8[s % 4].data_ptr(), W, u8=True)), 4)
        r["host_u8_ms"] = round(loop(det, depth, lambda s: det.submit(host8[s % 4])), 4)
        r["host_u8_fetch_ms"] = round(loop(det, depth, lambda s: det.submit(host8[s % 4]), True), 4)
        r["lanes_created"] = det.lanes()[1]
        print(json.dumps(r), flush=True)
    del det

# host-side costs per call (one lane, frames synchronous)
det = sift.Detector(cfg, lanes=1)
det.gpuWarmUpAndAllocate()
t_sub, t_wait, t_copy = [], [], []
for s in range(40):
    t0 = time.perf_counter()
    tk = det.submit(host8[s % 4])
    t1 = time.perf_counter()
    det.wait(tk)
    t2 = time.perf_counter()
    det.copyToHost(True)
    t3 = time.perf_counter()
    t_sub.append(t1 - t0), t_wait.append(t2 - t1), t_copy.append(t3 - t2)
buf = np.empty_like(host8[0])
t = time.perf_counter()
for _ in range(40):
    np.copyto(buf, host8[1])
t_memcpy = (time.perf_counter() - t) / 40
print(json.dumps({"host_costs_ms": {"submit_u8": round(np.median(t_sub) * 1e3, 4),
                                    "wait": round(np.median(t_wait) * 1e3, 4),
                                    "copyToHost_desc": round(np.median(t_copy) * 1e3, 4),
                                    "numpy_copy_2.3MB": round(t_memcpy * 1e3, 4),
                                    "keypoints": det.total_size}}), flush=True)

"""Blur phase timing from a -DSIFT_BLUR_STAMPS build (tools/ab_variant.sh):
C2 batch workload, summed s_memtime cycles per phase per tile, by radius.
    SIFT_HIP_LIB=ab/bstamps.so python tools/blur_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

B, W, H, N = 8, 1920, 1200, 5
cfg = sift.CudaSiftConfig(col_width=W, row_width=H, numOctaves=3, numFeatures=5000)
det = sift.Detector(cfg, device=0, batch=B)
det.gpuWarmUpAndAllocate()
buf = sift.DeviceArray.from_numpy(np.stack([sift.synth_frame(i, W, H) for i in range(B)]))
f = sift.lib().sift_hip_debug_blur_stamps
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
a = (ctypes.c_ulonglong * 192)()
det.detectBatchDevice(buf.value, B, W * 4, W * H * 4)
f(a)
for _ in range(N):
    det.detectBatchDevice(buf.value, B, W * 4, W * H * 4)
b = (ctypes.c_ulonglong * 192)()
f(b)
names = ["load+lds_write", "stage_barrier", "row_pass", "col_pass+store_issue", "store_drain"]
for r in range(32):
    d = [b[r * 6 + i] - a[r * 6 + i] for i in range(6)]
    if d[5]:
        print(r, {"tiles": d[5], **{n: round(d[i] / d[5]) for i, n in enumerate(names)}})

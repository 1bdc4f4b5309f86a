"""Descriptor phase timing from a -DSIFT_DESC_STAMPS build (tools/ab_variant.sh):
runs the C2 batch workload and prints the summed s_memtime cycles per phase
(setup / samples / epilogue) per keypoint.
    SIFT_HIP_LIB=ab/stamps.so python tools/desc_stamps.py"""
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
frames = np.stack([sift.synth_frame(i, W, H) for i in range(B)])
buf = sift.DeviceArray.from_numpy(frames)
lib = sift.lib()
f = lib.sift_hip_debug_desc_stamps
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
out0 = (ctypes.c_ulonglong * 8)()
det.detectBatchDevice(buf.value, B, W * 4, W * H * 4)
f(out0)
for _ in range(N):
    det.detectBatchDevice(buf.value, B, W * 4, W * H * 4)
out = (ctypes.c_ulonglong * 8)()
f(out)
d = [out[i] - out0[i] for i in range(8)]
kp = d[4]
print({"keypoints": kp, "workgroups": d[5], "cycles_per_kp": {"pre": d[0] / kp, "setup": d[1] / kp, "samples": d[2] / kp, "epilogue": d[3] / kp}})

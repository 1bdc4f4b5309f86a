"""Per-plane start times of the pyramid tail (diagnostic build -DSIFT_TAIL_DIAG=5
writes s_memtime of each plane into octave 0 / plane 0, which it corrupts):
    SIFT_HIP_LIB=ab/td5.so python tools/tail_stamps.py [W H]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (752, 480)
d = sift.Detector(sift.CudaSiftConfig(col_width=W, row_width=H, numFeatures=5000, upscale=False), device=0)
d.gpuWarmUpAndAllocate()
img = sift.synth_frame(0, W, H)
for _ in range(3):
    d.detectAndCompute(img)
p = d.debug_gaussian(0, 0).ravel().view(np.uint32)
t = p[0:2 * 40:2].astype(np.uint64) | (p[1:2 * 40:2].astype(np.uint64) << np.uint64(32))
n = int(np.argmax(t == 0)) if (t == 0).any() else len(t)
t = t[:n].astype(np.int64)
print("planes", n, "ticks between plane starts (s_memtime, ~100 MHz?):", list(np.diff(t)))

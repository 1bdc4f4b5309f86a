"""Run the C2 workload (or another configuration: --upscale --octaves 0 --features 0 is
OpenCV's default) for a few frames (no torch) -- a small target for rocprofv3."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=10)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1200)
ap.add_argument("--octaves", type=int, default=3)
ap.add_argument("--upscale", action="store_true")
ap.add_argument("--features", type=int, default=5000, help="numFeatures (0: keep all, OpenCV's default)")
ap.add_argument("--eager", action="store_true", help="timing mode: un-graphed launches")
ap.add_argument("--batch", type=int, default=1, help="frames per launch (sift_hip_set_batch)")
ap.add_argument("--exact", action="store_true", help="exact descriptor mode (SIFT_HIP_DESC_EXACT)")
ap.add_argument("--hash", action="store_true", help="print a digest of every frame's results (A/B builds must agree)")
a = ap.parse_args()
cfg = sift.CudaSiftConfig(col_width=a.width, row_width=a.height, numOctaves=a.octaves, upscale=a.upscale,
                          numFeatures=a.features)
det = sift.Detector(cfg, device=0, batch=a.batch, exact_descriptors=a.exact)
det.gpuWarmUpAndAllocate()
det.set_timing(a.eager)
img = sift.synth_frame(0, a.width, a.height)
if a.batch > 1:  # B copies of the frame, device-resident
    buf = sift.DeviceArray.from_numpy(np.ascontiguousarray(np.broadcast_to(img, (a.batch,) + img.shape)))
for _ in range(a.frames):
    if a.batch > 1:
        det.detectBatchDevice(buf.value, a.batch, a.width * 4, a.width * a.height * 4)
    else:
        det.detectAndCompute(img)
print("keypoints", det.total_size)
if a.hash:
    import hashlib
    h = hashlib.sha256()
    for i in range(det.batch_frames() if a.batch > 1 else 1):
        k3, f4, d = det.batch_copy_to_host(i) if a.batch > 1 else (det.copyToHost(), det.final_kpts, det.final_features,
                                                                   det.descriptors)[1:]
        for x in (k3, f4, d):
            h.update(np.ascontiguousarray(x).tobytes())
    print("results sha256", h.hexdigest()[:16])
if a.eager:
    for k, v in sorted(det.timing().items(), key=lambda kv: -kv[1]["ms"]):
        print(f"{k:16s} {v['ms'] / a.frames * 1e3:9.2f} us/frame  launches/frame {v['launches'] / a.frames:.0f}")

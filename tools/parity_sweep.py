"""Parity sweep beyond the test fixtures: fresh synthetic frames (seeds the
tests do not use) through the HIP path and the CPU oracle, keypoints compared
bit for bit and descriptor flips counted.

    python3 tools/parity_sweep.py [FRAMES_PER_CONFIG] [--exact] > gpurun_out/parity_sweep.json   (GPU box)

--exact: the exact descriptor mode (SIFT_HIP_DESC_EXACT), where every
descriptor byte must equal the oracle's (flips = 0).

Configurations: BASELINE C2 (1920x1200, 3 octaves, numFeatures 5000) and
OpenCV defaults (doubled base, keep all) at 752x480 (C1's frame).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import oracle_binding as oracle  # noqa: E402
import sift_amd as sift  # noqa: E402
from test_gpu_parity import gpu_keypoints, sort_keys  # noqa: E402

ARGS = [a for a in sys.argv[1:] if not a.startswith("--")]
EXACT = "--exact" in sys.argv[1:]
N = int(ARGS[0]) if ARGS else 10  # frames per configuration (seeds unused by the tests)
CONFIGS = [("C2", 1920, 1200, dict(upscale=False, numOctaves=3, numFeatures=5000), range(1000, 1000 + N)),
           ("C1 OpenCV defaults", 752, 480, dict(upscale=True, numOctaves=0, numFeatures=0), range(5000, 5000 + N))]


def main():
    rows, tot = [], {"frames": 0, "keypoints": 0, "keypoint_field_mismatches": 0, "entries": 0, "flips": 0,
                     "max_abs_diff": 0}
    for name, w, h, kw, seeds in CONFIGS:
        cfg = sift.CudaSiftConfig(col_width=w, row_width=h, **kw)
        det = sift.Detector(cfg, exact_descriptors=EXACT)
        det.gpuWarmUpAndAllocate()
        for seed in seeds:
            img = sift.synth_frame(seed, w, h)
            det.detectAndCompute(img)
            gk, gd, _ = gpu_keypoints(det)
            ok, od = oracle.detect_and_compute(img, oracle.from_config(cfg))
            row = {"config": name, "seed": seed, "gpu_keypoints": int(len(gk)), "oracle_keypoints": int(len(ok))}
            if len(gk) == len(ok):
                gs, os_ = gk[sort_keys(gk)], ok[sort_keys(ok)]
                mism = sum(int(np.count_nonzero(gs[f].view(np.uint32) != os_[f].view(np.uint32)))
                           for f in ("x", "y", "size", "angle", "response"))
                mism += int(np.count_nonzero(gs["octave"] != os_["octave"]))
                d = np.abs(gd[sort_keys(gk)] - od[sort_keys(ok)])
                row.update(keypoint_field_mismatches=mism, entries=int(d.size), flips=int(np.count_nonzero(d)),
                           max_abs_diff=float(d.max()) if d.size else 0.0)
                tot["keypoint_field_mismatches"] += mism
                tot["entries"] += int(d.size)
                tot["flips"] += int(np.count_nonzero(d))
                tot["max_abs_diff"] = max(tot["max_abs_diff"], row["max_abs_diff"])
            else:
                row["keypoint_field_mismatches"] = -1
                tot["keypoint_field_mismatches"] += 1
            tot["frames"] += 1
            tot["keypoints"] += int(len(gk))
            rows.append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
    tot["exact_fraction"] = 1.0 - tot["flips"] / max(1, tot["entries"])
    cmd = f"python3 tools/parity_sweep.py {N}" + (" --exact" if EXACT else "")
    json.dump({"command": cmd, "descriptor_mode": "exact" if EXACT else "fast", "total": tot, "frames": rows},
              sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

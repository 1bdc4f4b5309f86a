"""The descriptor parity bar shared by every GPU test that compares descriptors
with the CPU oracle.

Keypoints (position, size, angle, response, packed octave) are bit-exact; a
descriptor entry may differ from the oracle's by at most 1.  The 4x4x8
histogram is summed here in exact fixed point (order independent) while
OpenCV sums the same float contributions sequentially, so an entry whose
value x 512 / |v| lands within the float summation error of a .5 boundary
rounds the other way.  Measured on the GPU: up to 0.15 % of the entries of a
configuration (gpurun_out/descriptor_exact.txt on the box), so the bar is
99.8 % exact: a regression that doubles the flip rate fails it.
"""
import os

import numpy as np

DESC_MAX_ABS_DIFF = 1.0
DESC_EXACT_MIN = 0.998

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def record_exact(tag, diff):
    """Log the exact fraction and flip count (gpurun_out/ travels back from the GPU box)."""
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        mx = float(diff.max()) if diff.size else 0.0
        with open(os.path.join(out, "descriptor_exact.txt"), "a") as f:
            f.write(f"{tag}: exact {(diff == 0).mean() if diff.size else 1.0:.6f} flips {int((diff != 0).sum())} "
                    f"max {mx:.0f} n {diff.size}\n")


def assert_descriptor_bar(gd, od, tag=""):
    """gd, od: (n, 128) descriptors of the same keypoints in the same order."""
    diff = np.abs(np.asarray(gd, np.float32) - np.asarray(od, np.float32))
    record_exact(tag, diff)
    if diff.size == 0:
        return diff
    assert diff.max() <= DESC_MAX_ABS_DIFF, f"{tag} descriptor max |diff| {diff.max()}"
    exact = (diff == 0).mean()
    assert exact >= DESC_EXACT_MIN, f"{tag} exact fraction {exact:.6f} < {DESC_EXACT_MIN} ({int((diff != 0).sum())} flips)"
    return diff

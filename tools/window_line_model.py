"""Bytes the orientation windows must fetch, at cache-line granularity.

For the C2 frame (1920x1200, 3 octaves, numFeatures 5000) the oracle's
keypoints give each refined keypoint's gradient window ((2r+1)^2 samples, each
reading its 4 neighbours: a (2r+3)^2 - 4 pixel footprint).  Per 16-frame batch:
  algo      4 B x (2r+1)^2 per keypoint (DESIGN section 4's model)
  border    4 B x ((2r+3)^2 - 4): the footprint itself
  no-reuse  lines touched, summed over keypoints (every window fetched alone)
  union     distinct lines touched per plane (a perfect cache)
at 32/64/128-byte lines.  k_orientation's measured FETCH_SIZE x 2 sits at the
no-reuse figure when a frame's keypoints spread over all XCDs (round 4: 270.4
MB) and near the union with frames pinned to XCDs (round 5: 209.9 MB vs
192.1).  Usage: python tools/window_line_model.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "another-cuda-sift_amd")]
import numpy as np  # noqa: E402

import oracle_binding as o  # noqa: E402
import sift_amd as sift  # noqa: E402

W, H, NF = 1920, 1200, 16
img = sift.synth_frame(0, W, H)
k, _ = o.detect_and_compute(img, o.params(firstOctave=0, nOctaves=3, nfeatures=5000))
oct_ = k["octave"] & 255
layer = (k["octave"] >> 8) & 255
rad = np.round(4.5 * (k["size"] * 0.5 / 2.0 ** oct_)).astype(int)
r = np.round(k["y"] / 2.0 ** oct_).astype(int)
c = np.round(k["x"] / 2.0 ** oct_).astype(int)
pitch = {q: ((W >> q) + 63) // 64 * 64 for q in range(3)}
for lb in (32, 64, 128):
    seen, planes, summed, algo, border = set(), {}, 0, 0, 0
    for i in range(len(k)):
        key = (oct_[i], layer[i], r[i], c[i])
        if key in seen:  # extra orientation peaks share the refined keypoint's window
            continue
        seen.add(key)
        R = rad[i]
        algo += 4 * (2 * R + 1) ** 2
        border += 4 * ((2 * R + 3) ** 2 - 4)
        lines = planes.setdefault((oct_[i], layer[i]), set())
        for yy in range(r[i] - R - 1, r[i] + R + 2):
            b0 = (yy * pitch[oct_[i]] + c[i] - R - 1) * 4 // lb
            b1 = (yy * pitch[oct_[i]] + c[i] + R + 1) * 4 // lb
            summed += b1 - b0 + 1
            lines.update(range(b0, b1 + 1))
    union = sum(len(v) for v in planes.values())
    print(f"line {lb:3d} B: per {NF}-frame batch  algo {algo * NF / 1e6:.1f} MB  border {border * NF / 1e6:.1f} MB  "
          f"no-reuse {summed * lb * NF / 1e6:.1f} MB  union {union * lb * NF / 1e6:.1f} MB  ({len(seen)} windows/frame)")

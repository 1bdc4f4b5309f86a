"""Walk-cost model of the exact descriptor kernel (descriptor.hip
k_descriptor_exact) on real keypoints: the current owner layout (one wave per
keypoint, lane = (cell, orientation pair), 64-sample raster chunks) against the
review's alternative -- a chunk's walk split by cell row over two waves (lane =
(cell of the wave's two cell rows, orientation bin), 128-sample steps, each
wave computing the records of 64 of them).

The walk is the kernel's divergent part: per 32-sample half of a chunk the wave
loops until its busiest lane has walked all its hits, two hits per step
(kExactHits), so a half costs max over lanes of ceil(hits / 2) steps.  The
sample math (phase 1) costs the same per sample in both layouts.  Reported per
keypoint and in total: walk steps of the wave-time (what a full GPU's
throughput pays: both waves' steps) and of the latency (the slower wave per
step).  Samples (r0, c0, o0) follow OpenCV's calcSIFTDescriptor on the
oracle's own Gaussian planes and keypoints (C2 frame).

    python3 tools/exact_walk_cost_model.py [--every K] > profiles/round5/exact_walk_model.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "another-cuda-sift_amd")]
import oracle_binding as ob  # noqa: E402  (test infrastructure: CPU oracle)

D, NB = 4, 8


def fast_atan2_deg(dy, dx):
    """Degrees in [0, 360) (the model only needs the bin; float64 atan2)."""
    a = np.degrees(np.arctan2(dy, dx))
    return np.where(a < 0, a + 360.0, a)


def samples_of(kp, pyr, first_octave, L):
    """(r0, c0, o0) of the keypoint's window samples in raster order."""
    octv = int(kp["octave"]) & 255
    layer = (int(kp["octave"]) >> 8) & 255
    octv = octv if octv < 128 else octv - 256
    scale = 1.0 / (1 << octv) if octv >= 0 else float(1 << -octv)
    img = pyr[octv - first_octave][layer]
    rows, cols = img.shape
    size = np.float32(kp["size"]) * np.float32(scale)
    ptx, pty = int(np.round(kp["x"] * scale)), int(np.round(kp["y"] * scale))
    angle = np.float32(360.0) - np.float32(kp["angle"])
    if abs(angle - 360.0) < np.finfo(np.float32).eps:
        angle = np.float32(0)
    hist_width = np.float32(3.0) * np.float32(size * 0.5)
    radius = int(np.round(hist_width * 1.4142135623730951 * (D + 1) * 0.5))
    radius = min(radius, int(np.sqrt(cols * cols + rows * rows)))
    cos_t = np.float32(np.cos(angle * np.pi / 180)) / hist_width
    sin_t = np.float32(np.sin(angle * np.pi / 180)) / hist_width
    i, j = np.mgrid[-radius:radius + 1, -radius:radius + 1]
    c_rot = j * cos_t - i * sin_t
    r_rot = j * sin_t + i * cos_t
    rbin = r_rot + D / 2 - 0.5
    cbin = c_rot + D / 2 - 0.5
    r, c = pty + i, ptx + j
    ok = (rbin > -1) & (rbin < D) & (cbin > -1) & (cbin < D) & (r > 0) & (r < rows - 1) & (c > 0) & (c < cols - 1)
    r, c, rbin, cbin = r[ok], c[ok], rbin[ok], cbin[ok]  # row-major = raster order
    dx = img[r, c + 1] - img[r, c - 1]
    dy = img[r - 1, c] - img[r + 1, c]
    obin = (fast_atan2_deg(dy, dx) - angle) * (NB / 360.0)
    o0 = np.floor(obin).astype(np.int64) % NB
    return np.floor(rbin).astype(np.int64), np.floor(cbin).astype(np.int64), o0


def lane_masks(r0, c0, o0, per_bin, cell_rows):
    """Boolean (lanes, samples): which samples each lane walks."""
    out = []
    for ci in cell_rows:
        for cj in range(D):
            rc = np.isin(r0, (ci - 1, ci)) & np.isin(c0, (cj - 1, cj))
            if per_bin:  # lane owns bin b: samples with o0 in {b - 1, b}
                for b in range(NB):
                    out.append(rc & np.isin(o0, ((b - 1) % NB, b)))
            else:  # lane owns pair g: o0 in {2g - 1, 2g, 2g + 1}
                for g in range(4):
                    out.append(rc & np.isin(o0, ((2 * g - 1) % NB, 2 * g, 2 * g + 1)))
    return np.array(out)


def half_steps(m, balanced=False):
    """Walk steps of one wave over 32-sample halves: sum over halves of max over lanes of ceil(hits / 2)
    (balanced: the same hits spread evenly over the lanes, the bound of any re-assignment)."""
    n = m.shape[1]
    steps = 0
    for h0 in range(0, n, 32):
        hits = m[:, h0:h0 + 32].sum(axis=1)
        if balanced:
            steps += int(np.ceil(hits.sum() / len(hits) / 2))
        else:
            steps += int(np.max((hits + 1) // 2)) if len(hits) else 0
    return steps


def model(r0, c0, o0):
    n = len(r0)
    cur = split_tp = split_lat = bal = 0
    pair_all = lane_masks(r0, c0, o0, False, range(D))
    binA = lane_masks(r0, c0, o0, True, (0, 1))
    binB = lane_masks(r0, c0, o0, True, (2, 3))
    for k0 in range(0, n, 64):
        cur += half_steps(pair_all[:, k0:k0 + 64])
        bal += half_steps(pair_all[:, k0:k0 + 64], balanced=True)
    for k0 in range(0, n, 128):
        a, b = half_steps(binA[:, k0:k0 + 128]), half_steps(binB[:, k0:k0 + 128])
        split_tp += a + b
        split_lat += max(a, b)
    return n, cur, split_tp, split_lat, bal


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=4, help="model every K-th keypoint")
    a = ap.parse_args()
    W, H = 1920, 1200
    import sift_amd as sift  # synthetic frame generator of the bench (no GPU call)

    img = sift.synth_frame(0, W, H)
    p = ob.params(nfeatures=5000, firstOctave=0, nOctaves=3)
    kps, _ = ob.detect_and_compute(img, p)
    pyr = ob.gaussian_pyramid(img, p)
    tot = np.zeros(5, np.int64)
    rows = []
    for kp in kps[::a.every]:
        r0, c0, o0 = samples_of(kp, pyr, 0, 3)
        n, cur, tp, lat, bal = model(r0, c0, o0)
        tot += (n, cur, tp, lat, bal)
        rows.append((n, cur, tp, lat, bal))
    rows = np.array(rows)
    chunks = int(np.ceil(rows[:, 0] / 64).sum())
    print(json.dumps({
        "workload": f"C2 frame 0 (1920x1200, 3 octaves, numFeatures 5000), every {a.every}th of {len(kps)} oracle keypoints",
        "keypoints_modelled": int(len(rows)), "samples": int(tot[0]), "chunks_64": chunks,
        "walk_steps_current": int(tot[1]),
        "walk_steps_split_wave_time": int(tot[2]),
        "walk_steps_split_latency": int(tot[3]),
        "wave_time_ratio_split_over_current": round(float(tot[2] / tot[1]), 3),
        "latency_ratio_split_over_current": round(float(tot[3] / tot[1]), 3),
        "steps_per_chunk_current": round(float(tot[1] / chunks), 2),
        "walk_steps_current_if_balanced": int(tot[4]),
        "balance_efficiency_current": round(float(tot[4] / tot[1]), 3),
        "note": "walk steps = per 32-sample half, the busiest lane's ceil(hits / 2) (the kernel's divergent loop, 2 hits "
                "per step); current: lane = (cell, orientation pair), one wave, 64-sample chunks; split: lane = (cell, "
                "bin) over two waves by cell row, 128-sample steps; phase-1 sample math is the same per sample in both",
    }, indent=1))


if __name__ == "__main__":
    main()

"""Keypoint-set comparison for the OpenCV-tolerance ensemble.

Two detectAndCompute results of the same frame (HIP path vs an oracle build,
or two oracle builds) are paired keypoint by keypoint and their differences
summarised: count delta, unpaired keypoints, the refined integer grid index
(octave, layer, r, c), max |dx|, |dy|, |dsize|/size, |dangle|, response
relative difference, and descriptor flips.  tests/parity_bar.py holds the
tolerance these numbers are checked against; tools/oracle_ensemble.py
derives it over a frame sweep.

Test infrastructure (CPU, numpy/scipy only).
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import cKDTree

# Pairing radius in the (x, y, size, angle) embedding: two keypoints of one
# frame from different builds are the same extremum when they differ by
# far less than this (builds move a keypoint by < 1e-2 px); distinct extrema
# of one frame are farther apart (the 3x3x3 scan keeps them >= 1 octave px).
PAIR_RADIUS = 0.05


def _octave_byte(octave):
    o = octave.astype(np.int64) & 255
    return np.where(o >= 128, o - 256, o)


def grid_index(k):
    """(octave, layer, r, c) of each keypoint, as adjustLocalExtrema left it:
    the refined pixel is round(pt / 2^octave) because |xc|, |xr| < 0.5."""
    o = _octave_byte(k["octave"])
    layer = (k["octave"].astype(np.int64) >> 8) & 255
    scale = np.exp2(-o.astype(np.float64))
    r = np.rint(k["y"].astype(np.float64) * scale).astype(np.int64)
    c = np.rint(k["x"].astype(np.float64) * scale).astype(np.int64)
    return np.stack([o, layer, r, c], 1)


def _embed(k):
    a = np.deg2rad(k["angle"].astype(np.float64))
    # angle as a point on a circle of radius 10 (wrap at 0/360; 1e-3 deg ~ 2e-4)
    return np.stack([k["x"], k["y"], k["size"], 10 * np.cos(a), 10 * np.sin(a)], 1).astype(np.float64)


def pair(ka, kb):
    """Mutual nearest neighbours within PAIR_RADIUS: index arrays (ia, ib)."""
    if len(ka) == 0 or len(kb) == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    ea, eb = _embed(ka), _embed(kb)
    da, ja = cKDTree(eb).query(ea, distance_upper_bound=PAIR_RADIUS)
    db, jb = cKDTree(ea).query(eb, distance_upper_bound=PAIR_RADIUS)
    ia = np.nonzero(np.isfinite(da))[0]
    ia = ia[jb[ja[ia]] == ia]  # mutual
    return ia, ja[ia]


def compare(ka, da, kb, db):
    """Differences between two results of one frame (keypoints structured
    arrays with x, y, size, angle, response, octave; descriptors (n, 128))."""
    ia, ib = pair(ka, kb)
    a, b = ka[ia], kb[ib]
    out = {"n_a": int(len(ka)), "n_b": int(len(kb)), "paired": int(len(ia)),
           "unpaired_a": int(len(ka) - len(ia)), "unpaired_b": int(len(kb) - len(ib))}
    if len(ia):
        dang = np.abs(a["angle"].astype(np.float64) - b["angle"])
        dang = np.minimum(dang, 360.0 - dang)
        out.update(
            max_dx=float(np.abs(a["x"].astype(np.float64) - b["x"]).max()),
            max_dy=float(np.abs(a["y"].astype(np.float64) - b["y"]).max()),
            max_dsize_rel=float((np.abs(a["size"].astype(np.float64) - b["size"]) / b["size"]).max()),
            max_dangle=float(dang.max()),
            max_dresponse_rel=float((np.abs(a["response"].astype(np.float64) - b["response"]) /
                                     np.maximum(b["response"], 1e-30)).max()),
            bit_identical=int(sum(np.all([a[f].view(np.uint32) == b[f].view(np.uint32)
                                          for f in ("x", "y", "size", "angle", "response")], 0)
                                  & (a["octave"] == b["octave"]))),
            grid_index_mismatch=int(np.count_nonzero(np.any(grid_index(a) != grid_index(b), 1))),
            octave_layer_mismatch=int(np.count_nonzero((a["octave"] & 0xFFFF) != (b["octave"] & 0xFFFF))),
        )
        if da is not None and db is not None:
            d = np.abs(np.asarray(da, np.float32)[ia] - np.asarray(db, np.float32)[ib])
            out.update(desc_entries=int(d.size), desc_flips=int(np.count_nonzero(d)), desc_max_abs=float(d.max()))
    return out


def merge(rows):
    """Worst case / totals over per-frame compare() rows."""
    tot = {"frames": len(rows)}
    for k in ("n_a", "n_b", "paired", "unpaired_a", "unpaired_b", "bit_identical", "grid_index_mismatch",
              "octave_layer_mismatch", "desc_entries", "desc_flips"):
        tot[k] = int(sum(r.get(k, 0) for r in rows))
    for k in ("max_dx", "max_dy", "max_dsize_rel", "max_dangle", "max_dresponse_rel", "desc_max_abs"):
        tot[k] = float(max([r.get(k, 0.0) for r in rows] or [0.0]))
    tot["max_count_delta"] = int(max([abs(r["n_a"] - r["n_b"]) for r in rows] or [0]))
    tot["max_unpaired_frac"] = float(max([max(r["unpaired_a"], r["unpaired_b"]) / max(1, min(r["n_a"], r["n_b"]))
                                          for r in rows] or [0.0]))
    tot["desc_flip_rate"] = tot["desc_flips"] / max(1, tot["desc_entries"])
    tot["max_frame_flip_rate"] = float(max([r.get("desc_flips", 0) / max(1, r.get("desc_entries", 0))
                                            for r in rows] or [0.0]))
    return tot

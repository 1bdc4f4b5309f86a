"""OpenCV interop, mirroring the reference's
cvUtils/Conversion.hh:12-70 (``OpencvUtils::localKptToCvKpt``,
``descriptorToCvMat``, ``cvtMatchToDMatch``).  The field mapping is plain
numpy so it is usable (and tested) without OpenCV; the ``cv2`` object builders
import cv2 lazily and raise ImportError where OpenCV is absent.
"""
from typing import List, Sequence

import numpy as np


def keypoint_fields(final_kpts: np.ndarray, final_features: np.ndarray, size: int = -1) -> dict:
    """Conversion.cc:21-42 field by field: pt = kpts[:, :2], octave = int(features.x),
    size = features.y, response = features.z, angle = features.w."""
    k = np.asarray(final_kpts, np.float32).reshape(-1, 3)
    f = np.asarray(final_features, np.float32).reshape(-1, 4)
    if len(k) != len(f):
        raise ValueError("kpts and features differ in length")
    n = len(k) if size < 0 else min(size, len(k))
    return {"x": k[:n, 0], "y": k[:n, 1], "octave": f[:n, 0].astype(np.int64).astype(np.int32),
            "size": f[:n, 1], "response": f[:n, 2], "angle": f[:n, 3]}


def descriptor_matrix(descriptors: np.ndarray, num_pts: int) -> np.ndarray:
    """ConversionImpl.hpp:66-82: row-major 128-wide descriptors -> float32 (n, 128)."""
    d = np.asarray(descriptors).reshape(-1, 128)
    n = min(num_pts, len(d))
    return d[:n].astype(np.float32)


def dmatch_triples(match: Sequence[int]) -> List[tuple]:
    """Conversion.cc:44-58: (queryIdx, trainIdx, distance 0) for every match != -1."""
    return [(i, int(m), 0.0) for i, m in enumerate(match) if m != -1]


def to_cv_keypoints(final_kpts, final_features, size: int = -1):
    import cv2

    f = keypoint_fields(final_kpts, final_features, size)
    out = []
    for i in range(len(f["x"])):
        kp = cv2.KeyPoint(float(f["x"][i]), float(f["y"][i]), float(f["size"][i]), float(f["angle"][i]),
                          float(f["response"][i]), int(f["octave"][i]))
        out.append(kp)
    return out


def to_cv_dmatches(match: Sequence[int]):
    import cv2

    return [cv2.DMatch(q, t, d) for q, t, d in dmatch_triples(match)]

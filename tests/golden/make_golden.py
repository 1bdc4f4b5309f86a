"""Generate the committed golden fixtures (run in the build container).

    python tests/golden/make_golden.py

Inputs
  * camera256: the central 256x256 crop of scikit-image's `camera.png` (CC0 per
    skimage/data/__init__.py; present in this container only, so the crop itself
    is stored in the fixture).
  * synth: sha256 of sift_amd.synth_frame for a few seeds/sizes (pins the
    in-repo PCG32 frame generator shared by tests and bench.py).
Outputs: the CPU oracle (oracle/sift_oracle.cpp, an OpenCV 4.x SIFT
restatement) on those inputs: Gaussian taps, per-plane pyramid checksums,
3x3x3 candidates, keypoints + descriptors for two configurations, and a knn-2
match of the crop against its 90-degree rotation.

OpenCV itself is absent, so these fixtures pin the oracle
against regressions and give the GPU tests fixed inputs/outputs; they do not
pin the oracle to OpenCV ("parity unpinned").
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "another-cuda-sift_amd")]
import oracle_binding as oracle  # noqa: E402

CAMERA = "/opt/conda/lib/python3.9/site-packages/skimage/data/camera.png"
SIGMAS = [0.5, 1.0, 1.2262735, 1.5450173, 1.6, 1.9465878, 2.4525471, 3.0900346]
CONFIGS = {
    # name: oracle params (OpenCV defaults except where noted)
    "default": dict(),                                  # firstOctave -1 (doubled base), nfeatures 0
    "base_n60": dict(firstOctave=0, nfeatures=60),      # reference default upscale=false; retainBest active
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def camera_crop():
    from PIL import Image

    im = np.asarray(Image.open(CAMERA).convert("L"))
    h, w = im.shape
    y0, x0 = (h - 256) // 2, (w - 256) // 2
    return np.ascontiguousarray(im[y0:y0 + 256, x0:x0 + 256])


def main():
    crop = camera_crop()
    img = crop.astype(np.float32)
    out = {"camera256": crop}
    for s in SIGMAS:
        out[f"taps_{s!r}"] = oracle.gaussian_taps(s)
    meta = {"sigmas": SIGMAS, "configs": CONFIGS, "pyramid_sha": {}}
    for name, kw in CONFIGS.items():
        p = oracle.params(**kw)
        pyr = oracle.gaussian_pyramid(img, p)
        meta["pyramid_sha"][name] = [[sha(pl) for pl in planes] for planes in pyr]
        out[f"{name}_extrema"] = oracle.extrema(img, p)
        k, d = oracle.detect_and_compute(img, p, threads=8)
        out[f"{name}_kpts"] = k
        out[f"{name}_desc"] = d.astype(np.uint8)
    rot = np.ascontiguousarray(np.rot90(img))
    p = oracle.params()
    _, da = oracle.detect_and_compute(img, p, threads=8)
    _, db = oracle.detect_and_compute(rot, p, threads=8)
    idx, dist = oracle.knn2(da, db, threads=8)
    out["rot90_knn_idx"], out["rot90_knn_dist"] = idx, dist
    np.savez_compressed(os.path.join(HERE, "camera256.npz"), **out)

    import sift_amd

    synth = {}
    for seed, w, h in [(0, 320, 240), (1, 257, 191), (7, 1920, 1200)]:
        synth[f"{seed}_{w}x{h}"] = sha(sift_amd.synth_frame(seed, w, h))
    meta["synth_sha"] = synth
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("keypoints:", {n: len(out[f"{n}_kpts"]) for n in CONFIGS}, "rot90 matches",
          int(((dist[:, 0] < 0.8 * dist[:, 1])).sum()))


if __name__ == "__main__":
    main()

"""The stage-dump replay checker (tests/stage_check.py) on CPU: a dump written
from the oracle's own stage outputs in the library's file format passes, and
a dump with one plane pixel, one candidate or one descriptor entry changed
fails at exactly that stage."""
import json
import os

import numpy as np

import stage_check


def _write_dump(dirname, oracle, img, cfg):
    p = oracle.params(cfg["numFeatures"], cfg["numOctaveLayers"], cfg["contrastThreshould"], cfg["edgeThreshould"],
                      cfg["sigma"], -1 if cfg["upscale"] else 0, cfg["numOctaves"])
    h, w = img.shape
    pyr = oracle.gaussian_pyramid(img, p)
    cand = oracle.extrema(img, p)
    kp, desc = oracle.detect_and_compute(img, p)
    os.makedirs(dirname, exist_ok=True)
    img.astype(np.float32).tofile(os.path.join(dirname, "input.f32"))
    for o, planes in enumerate(pyr):
        for l in range(planes.shape[0]):
            planes[l].tofile(os.path.join(dirname, f"gauss_o{o}_l{l}.f32"))
    cand[::-1].astype(np.int32).tofile(os.path.join(dirname, "candidates.i32"))  # order is not part of the contract
    k3 = np.stack([kp["x"], kp["y"], ((kp["octave"] >> 8) & 255).astype(np.float32)], 1).astype(np.float32)
    f4 = np.stack([kp["octave"].astype(np.float32), kp["size"], kp["response"], kp["angle"]], 1).astype(np.float32)
    k3.tofile(os.path.join(dirname, "kpts3.f32"))
    f4.tofile(os.path.join(dirname, "feats4.f32"))
    desc.astype(np.float16).tofile(os.path.join(dirname, "desc.f16"))
    meta = {"format": "sift_hip stage dump 1", "frame": 0, "width": w, "height": h, "config": cfg,
            "octaves": [[pl.shape[2], pl.shape[1]] for pl in pyr], "planes_per_octave": pyr[0].shape[0],
            "candidates": len(cand), "keypoints": len(kp)}
    with open(os.path.join(dirname, "meta.json"), "w") as f:
        json.dump(meta, f)


def test_stage_check_on_oracle_dump(sift, oracle, tmp_path):
    cfg = {"numFeatures": 0, "numOctaveLayers": 3, "contrastThreshould": 0.04, "edgeThreshould": 10.0, "sigma": 1.6,
           "upscale": 0, "numOctaves": 0}
    img = sift.synth_frame(4, 160, 120)
    d = str(tmp_path / "dump")
    _write_dump(d, oracle, img, cfg)
    res = stage_check.check_oracle(stage_check.load(d))
    assert all(v for v in res.values() if isinstance(v, bool)), res
    assert res["descriptor_exact"] == 1.0

    # one Gaussian pixel off by an ulp: only the plane stage fails
    path = os.path.join(d, "gauss_o1_l3.f32")
    g = np.fromfile(path, np.float32)
    g2 = g.copy()
    g2.view(np.uint32)[7] += 1
    g2.tofile(path)
    res = stage_check.check_oracle(stage_check.load(d))
    assert not res["gaussian_planes_bitexact"] and res["candidates_exact"] and res["keypoints_bitexact"]
    g.tofile(path)

    # a descriptor entry off by 2: the descriptor bar fails
    path = os.path.join(d, "desc.f16")
    desc = np.fromfile(path, np.float16)
    desc2 = desc.copy()
    desc2[5] = desc2[5] + 2
    desc2.tofile(path)
    res = stage_check.check_oracle(stage_check.load(d))
    assert res["keypoints_bitexact"] and not res["descriptors_within_bar"]
    desc.tofile(path)

    # a missing candidate: the candidate stage fails
    path = os.path.join(d, "candidates.i32")
    c = np.fromfile(path, np.int32)
    c[:-4].tofile(path)
    res = stage_check.check_oracle(stage_check.load(d))
    assert not res["candidates_exact"] and res["gaussian_planes_bitexact"]

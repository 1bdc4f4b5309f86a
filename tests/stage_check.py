"""Replay of a stage dump (Detector::setDataGen / sift_hip_set_datagen).

The reference's setDataGen writes each stage's octave-0 inputs and expected
outputs (/root/reference/sift_cuda/interface/Detector.cu:145-229,
sift_cuda/perf/PerfData.cuh:12-155) and tool/perf.cu:16-113 re-runs each
stage on them, comparing with HostInterface.cu's rules (exact floats for
blur / resize / DoG / peaks / refine / orientation, |diff| <= 1 for
descriptors).  This build's dump is the whole frame (meta.json + raw arrays,
layouts in meta.json); this checker replays it two ways:

  * against the CPU oracle (test infrastructure): every Gaussian plane
    bit-exact, the 3x3x3 candidate set exact, keypoints bit-exact, descriptors
    within the parity bar (parity_bar.py);
  * against this library (--gpu): the dumped input through a fresh detector
    gives the dumped planes, keypoints and descriptors bit for bit (a kernel
    regression check across builds or boxes).

    python tests/stage_check.py DIR [--gpu]      (exit status 1 on a mismatch)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load(dirname):
    with open(os.path.join(dirname, "meta.json")) as f:
        meta = json.load(f)
    w, h = meta["width"], meta["height"]
    rd = lambda name, dt: np.fromfile(os.path.join(dirname, name), dt)
    d = {"meta": meta, "input": rd("input.f32", np.float32).reshape(h, w)}
    d["gauss"] = [[rd(f"gauss_o{o}_l{l}.f32", np.float32).reshape(oh, ow) for l in range(meta["planes_per_octave"])]
                  for o, (ow, oh) in enumerate(meta["octaves"])]
    d["candidates"] = rd("candidates.i32", np.int32).reshape(-1, 4)
    d["kpts3"] = rd("kpts3.f32", np.float32).reshape(-1, 3)
    d["feats4"] = rd("feats4.f32", np.float32).reshape(-1, 4)
    d["desc"] = rd("desc.f16", np.float16).reshape(-1, 128)
    return d


def _keys(k3, f4):
    """Keypoints as (x, y, size, angle, response, octave) rows."""
    return np.stack([k3[:, 0], k3[:, 1], f4[:, 1], f4[:, 3], f4[:, 2], f4[:, 0]], 1)


def check_oracle(d):
    """Stage-by-stage parity of a dump with the CPU oracle.  Returns a dict of
    per-stage results; every value must be True for the dump to pass."""
    sys.path.insert(0, HERE)
    import oracle_binding as oracle
    from parity_bar import DESC_EXACT_MIN, DESC_MAX_ABS_DIFF

    c = d["meta"]["config"]
    p = oracle.params(c["numFeatures"], c["numOctaveLayers"], c["contrastThreshould"], c["edgeThreshould"], c["sigma"],
                      -1 if c["upscale"] else 0, c["numOctaves"])
    img = d["input"]
    out = {}
    pyr = oracle.gaussian_pyramid(img, p)
    out["octaves"] = len(pyr) == len(d["gauss"])
    out["gaussian_planes_bitexact"] = out["octaves"] and all(
        np.array_equal(g.view(np.uint32), o.view(np.uint32))
        for planes, ops in zip(d["gauss"], pyr) for g, o in zip(planes, ops))
    oc = oracle.extrema(img, p)
    gc = d["candidates"]
    out["candidates_exact"] = gc.shape == oc.shape and np.array_equal(gc[np.lexsort(gc.T[::-1])],
                                                                      oc[np.lexsort(oc.T[::-1])])
    ok, od = oracle.detect_and_compute(img, p)
    gk = _keys(d["kpts3"], d["feats4"])
    o = np.stack([ok["x"], ok["y"], ok["size"], ok["angle"], ok["response"], ok["octave"].astype(np.float32)], 1)
    same = len(gk) == len(o)
    if same:
        gi, oi = np.lexsort(gk.T[::-1]), np.lexsort(o.T[::-1])
        same = np.array_equal(gk[gi].view(np.uint32), o[oi].view(np.uint32))
        diff = np.abs(d["desc"].astype(np.float32)[gi] - od[oi])
        out["descriptor_max_diff"] = float(diff.max()) if diff.size else 0.0
        out["descriptor_exact"] = float((diff == 0).mean()) if diff.size else 1.0
        out["descriptors_within_bar"] = bool(out["descriptor_max_diff"] <= DESC_MAX_ABS_DIFF
                                             and out["descriptor_exact"] >= DESC_EXACT_MIN)
    else:
        out["descriptors_within_bar"] = False
    out["keypoints_bitexact"] = bool(same)
    return out


def check_gpu(d):
    """The dumped input through a fresh detector: the dump's planes, candidates,
    keypoints and descriptors again, bit for bit."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "another-cuda-sift_amd"))
    import sift_amd as sift

    m, c = d["meta"], d["meta"]["config"]
    cfg = sift.CudaSiftConfig(col_width=m["width"], row_width=m["height"], numFeatures=c["numFeatures"],
                              numOctaveLayers=c["numOctaveLayers"], contrastThreshould=c["contrastThreshould"],
                              edgeThreshould=c["edgeThreshould"], sigma=c["sigma"], upscale=bool(c["upscale"]),
                              numOctaves=c["numOctaves"])
    det = sift.Detector(cfg)
    det.gpuWarmUpAndAllocate()
    det.detectAndCompute(d["input"])
    det.copyToHost(True)
    out = {"gaussian_planes": all(np.array_equal(det.debug_gaussian(o, l).view(np.uint32), g.view(np.uint32))
                                  for o, planes in enumerate(d["gauss"]) for l, g in enumerate(planes))}
    gc = det.debug_candidates()
    dc = d["candidates"]
    out["candidates"] = gc.shape == dc.shape and np.array_equal(gc[np.lexsort(gc.T[::-1])], dc[np.lexsort(dc.T[::-1])])
    out["keypoints"] = np.array_equal(det.final_kpts.view(np.uint32), d["kpts3"].view(np.uint32)) and np.array_equal(
        det.final_features.view(np.uint32), d["feats4"].view(np.uint32))
    out["descriptors"] = np.array_equal(det.descriptors.view(np.uint16), d["desc"].view(np.uint16))
    return out


def main(argv):
    d = load(argv[1])
    res = {"oracle": check_oracle(d)}
    if "--gpu" in argv:
        import torch  # noqa: F401  (one HIP runtime per process: torch's, loaded first)

        res["gpu_replay"] = check_gpu(d)
    print(json.dumps(res, indent=1))
    ok = all(v for part in res.values() for k, v in part.items() if isinstance(v, bool))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv))

"""Replay of a stage dump (Detector::setDataGen / sift_hip_set_datagen).

The reference's setDataGen writes each stage's octave-0 inputs and expected
outputs (/root/reference/sift_cuda/interface/Detector.cu:145-229,
sift_cuda/perf/PerfData.cuh:12-155) and tool/perf.cu:16-113 re-runs each
stage on them, comparing with HostInterface.cu's rules (exact floats for
blur / resize / DoG / peaks / refine / orientation, |diff| <= 1 for
descriptors).  This build's dump is the whole frame (meta.json + raw arrays,
layouts in meta.json) plus the keypoint stages' device records; this checker
replays it three ways:

  * against the CPU oracle (test infrastructure): every Gaussian plane
    bit-exact, the 3x3x3 candidate set exact, keypoints bit-exact, descriptors
    within the parity bar (parity_bar.py);
  * against this library, whole frame (--gpu): the dumped input through a
    fresh detector gives the dumped planes, keypoints and descriptors bit for
    bit (a kernel regression check across builds or boxes);
  * against this library, ONE stage at a time (--stage S|all; S in
    pyramid, extrema, refine, orientation, order, descriptor): the stage's
    kernels alone on the dump's recorded input of that stage
    (sift_hip_replay_stage, as tool/perf.cu:43-100 runs HostInterface's
    run<Stage>), their output equal to the dump's -- bit for bit, as sets
    where the device appends with atomics (candidates, refined and oriented
    records).

    python tests/stage_check.py DIR [--gpu] [--stage S|all]   (exit status 1 on a mismatch)
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


STAGES = ("pyramid", "extrema", "refine", "orientation", "order", "descriptor")
# Outputs of each stage (the dump's file names) and how they compare:
# "exact" byte for byte, "rows" as sets of fixed-size records (appended by
# device atomics in any order).
STAGE_OUTPUTS = {
    "pyramid": None,  # every gauss_o<o>_l<l>.f32
    "extrema": [("candidates.i32", "rows", 16)],
    "refine": [("refined.rec", "rows", 32)],
    "orientation": [("oriented.rec", "rows", 32)],
    "order": [("kpts3.f32", "exact", 0), ("feats4.f32", "exact", 0), ("jobs.rec", "exact", 0)],
    "descriptor": [("desc.f16", "exact", 0)],
}


def _same_file(a, b, how, rec):
    x, y = np.fromfile(a, np.uint8), np.fromfile(b, np.uint8)
    if how == "exact" or x.size != y.size:
        return x.size == y.size and bool(np.array_equal(x, y))
    xr, yr = x.view(np.uint32).reshape(-1, rec // 4), y.view(np.uint32).reshape(-1, rec // 4)
    return bool(np.array_equal(xr[np.lexsort(xr.T[::-1])], yr[np.lexsort(yr.T[::-1])]))


def check_stages(dirname, stages=STAGES, det=None, out_root=None):
    """Each stage's kernels alone on the dump's recorded input
    (Detector.replayStage); {stage: True} where the outputs equal the dump's."""
    import tempfile

    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "another-cuda-sift_amd"))
    import sift_amd as sift

    d = load(dirname)
    m, c = d["meta"], d["meta"]["config"]
    if det is None:
        cfg = sift.CudaSiftConfig(col_width=m["width"], row_width=m["height"], numFeatures=c["numFeatures"],
                                  numOctaveLayers=c["numOctaveLayers"], contrastThreshould=c["contrastThreshould"],
                                  edgeThreshould=c["edgeThreshould"], sigma=c["sigma"], upscale=bool(c["upscale"]),
                                  numOctaves=c["numOctaves"])
        det = sift.Detector(cfg)
        det.gpuWarmUpAndAllocate()
    out_root = out_root or tempfile.mkdtemp(prefix="sift_replay_")
    res = {}
    for st in stages:
        out = os.path.join(out_root, st)
        det.replayStage(dirname, st, out)
        if STAGE_OUTPUTS[st] is None:
            names = [f"gauss_o{o}_l{l}.f32" for o in range(len(m["octaves"])) for l in range(m["planes_per_octave"])]
            res[st] = all(_same_file(os.path.join(dirname, n), os.path.join(out, n), "exact", 0) for n in names)
        else:
            res[st] = all(_same_file(os.path.join(dirname, n), os.path.join(out, n), how, rec)
                          for n, how, rec in STAGE_OUTPUTS[st])
    return res


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
        res["gpu_replay"] = check_gpu(d)
    if "--stage" in argv:
        st = argv[argv.index("--stage") + 1]
        res["stage_replay"] = check_stages(argv[1], STAGES if st == "all" else (st,))
    print(json.dumps(res, indent=1))
    ok = all(v for part in res.values() for k, v in part.items() if isinstance(v, bool))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv))

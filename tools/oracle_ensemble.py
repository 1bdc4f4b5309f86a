"""OpenCV-tolerance ensemble (CPU only): the same frames through the three
builds of the oracle (oracle/Makefile) -- "pinned" (the HIP path's bit-exact
pin), "avx2-fma" and "avx512-fma" (OpenCV's AVX2 / AVX-512 dispatch as GCC
compiles it: SIMD bodies + scalar tails, sift.simd.hpp contracted) -- and the
spread between them: candidate sets, keypoint counts, refined grid indices,
sub-pixel x/y, size, angle, response and descriptor flips.  The tolerance
tests/parity_bar.py states for "equal to OpenCV" is the envelope of this
spread.

    python3 tools/oracle_ensemble.py [FRAMES_PER_CONFIG] > profiles/round3/oracle_ensemble.json

Frames: the parity sweep's configurations and seeds (tools/parity_sweep.py):
C2 (1920x1200, 3 octaves, numFeatures 5000) seeds 1000.., and OpenCV defaults
at 752x480 (C1's frame) seeds 5000...
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import ensemble  # noqa: E402
import oracle_binding as oracle  # noqa: E402
import sift_amd as sift  # noqa: E402  (synth_frame only: CPU code in libsift_hip.so)

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
THREADS = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
VARIANTS = ["pinned", "avx2-fma", "avx512-fma"]
PAIRS = [("pinned", "avx2-fma"), ("pinned", "avx512-fma"), ("avx2-fma", "avx512-fma")]
CONFIGS = [("C2", 1920, 1200, dict(nfeatures=5000, firstOctave=0, nOctaves=3), range(1000, 1000 + N)),
           ("C1 OpenCV defaults", 752, 480, dict(nfeatures=0, firstOctave=-1, nOctaves=0), range(5000, 5000 + N))]


def main():
    t0 = time.time()
    out = {"command": f"python3 tools/oracle_ensemble.py {N}", "variants": VARIANTS, "configs": {}}
    for name, w, h, kw, seeds in CONFIGS:
        p = oracle.params(**kw)
        rows = {f"{a} vs {b}": [] for a, b in PAIRS}
        cand_diff = 0
        for seed in seeds:
            img = sift.synth_frame(seed, w, h)
            cands = [oracle.extrema(img, p, variant=v) for v in VARIANTS]
            s0 = {tuple(q) for q in cands[0]}
            for c in cands[1:]:
                cand_diff += len(s0.symmetric_difference({tuple(q) for q in c}))
            res = {v: oracle.detect_and_compute(img, p, threads=THREADS, variant=v) for v in VARIANTS}
            for a, b in PAIRS:
                r = ensemble.compare(res[a][0], res[a][1], res[b][0], res[b][1])
                r["seed"] = seed
                rows[f"{a} vs {b}"].append(r)
            print(f"{name} seed {seed}: " + ", ".join(f"{v}={len(res[v][0])}" for v in VARIANTS)
                  + f" ({time.time() - t0:.0f}s)", file=sys.stderr, flush=True)
        out["configs"][name] = {
            "frame": f"{w}x{h}", "params": kw, "frames": len(seeds),
            "candidate_symmetric_difference": cand_diff,
            "pairs": {k: {"total": ensemble.merge(v),
                          "frames_with_count_delta": int(sum(r["n_a"] != r["n_b"] for r in v))}
                      for k, v in rows.items()},
        }
    out["seconds"] = round(time.time() - t0, 1)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

"""Matcher parity sweep beyond the tests: random ragged pair sizes (1..3000
rows, duplicated rows for ties) through the single-pair HIP matcher, top-2
indices and squared distances against the oracle's knn-2.

    python3 tools/match_sweep.py [PAIRS] > gpurun_out/match_sweep.json   (GPU box)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import oracle_binding as oracle  # noqa: E402
import sift_amd as sift  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 60


def main():
    rng = np.random.default_rng(20261016)
    m = sift.Matcher(3000, 3000, max_pairs=1)
    rows, bad = [], 0
    for k in range(P):
        nq, nt = (int(x) for x in rng.integers(1, 3001, 2))
        hi = int(rng.choice([8, 32, 256]))  # small ranges: many equal distances
        q = rng.integers(0, hi, (nq, 128)).astype(np.float32)
        t = rng.integers(0, hi, (nt, 128)).astype(np.float32)
        if nt > 4:
            t[rng.integers(0, nt, nt // 4)] = t[rng.integers(0, nt, nt // 4)]  # duplicate train rows (ties)
        dq = sift.DeviceArray.from_numpy(np.ascontiguousarray(q.astype(np.float16)))
        dt = sift.DeviceArray.from_numpy(np.ascontiguousarray(t.astype(np.float16)))
        idx2, d2 = sift.DeviceArray(nq * 8), sift.DeviceArray(nq * 8)
        m.match_batched([dq.value], [nq], [dt.value], [nt], idx2_ptr=idx2.value, d2_ptr=d2.value)
        gi = idx2.to_numpy(np.int32, (nq, 2))
        gd = d2.to_numpy(np.float32, (nq, 2))
        oi, od = oracle.knn2(q, t)
        ok_i = bool(np.array_equal(gi, oi))
        ok_d = bool(np.array_equal(np.sqrt(gd).astype(np.float32), od))
        bad += not (ok_i and ok_d)
        row = {"nq": nq, "nt": nt, "value_range": hi, "indices_exact": ok_i, "distances_exact": ok_d}
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    json.dump({"command": f"python3 tools/match_sweep.py {P}", "pairs": P, "pairs_not_exact": bad, "rows": rows},
              sys.stdout, indent=1)
    print()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

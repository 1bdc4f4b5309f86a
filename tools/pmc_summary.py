"""Summarise tools/pmc.sh output into one JSON (committed under profiles/).

    python tools/pmc_summary.py TAG > profiles/<round>/pmc_summary.json

Per kernel name and grid size: dispatch count, mean of every counter per
dispatch.  FETCH_SIZE / WRITE_SIZE are KiB per dispatch as rocprofv3 reports
them; the calibration section gives the measured counter/true-byte ratios of
4-B and 16-B per-lane streaming copies (tools/hbm_calib.hip, 512 MiB each way),
which bench.py uses to correct FETCH_SIZE/WRITE_SIZE (MI355X_MICROARCH.md HBM
section: only 16-B/lane reads are documented, at exactly 1/2).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern):
    rows = []
    for f in glob.glob(pattern):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def main(tag, out_dir="gpurun_out"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(out_dir, f"{tag}_p*", "*counter_collection.csv"))):
        for r in load(f):
            key = (r["Kernel_Name"].split("(")[0][:80], int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = []
    for (name, grid), ctrs in sorted(acc.items()):
        e = {"kernel": name, "grid_size": grid}
        for c, v in sorted(ctrs.items()):
            e[c] = round(sum(v) / len(v), 3)
            e["dispatches"] = len(v)
        kernels.append(e)
    calib = {}
    true_kib = 512 * 1024
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for r in load(os.path.join(out_dir, f"{tag}_calib_{c}", "*counter_collection.csv")):
            if r["Counter_Name"] != c:
                continue
            k = r["Kernel_Name"].split("(")[0]
            calib.setdefault(f"{k}:{c}", []).append(float(r["Counter_Value"]) / true_kib)
    calib = {k: round(sum(v) / len(v), 4) for k, v in calib.items()}
    json.dump({"tag": tag, "units": "counter values per dispatch; FETCH/WRITE_SIZE in KiB",
               "calibration_counter_over_true_bytes": calib, "kernels": kernels}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise tools/pmc.sh output into one JSON (committed under profiles/).

    python tools/pmc_summary.py TAG > profiles/<round>/pmc_summary.json

Per kernel name and grid size, over the profiled frames' dispatches only
(profiled_rows drops the handle's warm-up): dispatch count, mean of every
counter per dispatch.  FETCH_SIZE / WRITE_SIZE are KiB per dispatch as rocprofv3 reports
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


def profiled_rows(rows):
    """The dispatches of the profiled frames only.  Every pipeline run ends with
    its k_descriptor dispatch; the handle's warm-up replays its batch graphs
    and then its single-frame graphs, so the profiled batches are the trailing
    runs whose first dispatch has the last run's (kernel, grid).  Single-frame
    warm-up dispatches share some (kernel, grid) groups with batch launches
    (k_orientation's grid), so filtering the summary by dispatch counts
    afterwards cannot separate them."""
    rows = sorted(rows, key=lambda r: (r["Counter_Name"], int(r["Dispatch_Id"])))
    out = []
    for _, grp in groupby_counter(rows):
        sift = [r for r in grp if "sift_amd::" in r["Kernel_Name"]]
        runs, cur = [], []
        for r in sift:
            cur.append(r)
            if "k_descriptor" in r["Kernel_Name"]:
                runs.append(cur)
                cur = []
        if not runs:
            continue
        sig = lambda run: (run[0]["Kernel_Name"], run[0]["Grid_Size"])  # noqa: E731
        k = len(runs) - 1
        while k > 0 and sig(runs[k - 1]) == sig(runs[-1]):
            k -= 1
        for run in runs[k:]:
            out += run
    return out


def groupby_counter(rows):
    groups = defaultdict(list)
    for r in rows:
        groups[r["Counter_Name"]].append(r)
    return sorted(groups.items())


def main(tag, out_dir="gpurun_out"):
    acc = defaultdict(lambda: defaultdict(list))
    runs = {}
    for f in sorted(glob.glob(os.path.join(out_dir, f"{tag}_p*", "*counter_collection.csv"))):
        rows = profiled_rows(load(f))
        for r in rows:
            key = (r["Kernel_Name"].split("(")[0][:80], int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if rows:
            runs[os.path.basename(os.path.dirname(f))] = sum("k_descriptor" in r["Kernel_Name"] for r in rows) // max(
                1, len({r["Counter_Name"] for r in rows}))
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
               "profiled_only": True,
               "note": "dispatches of the profiled frames only (the handle's warm-up runs are dropped, profiled_rows)",
               "profiled_runs_per_pass": runs,
               "calibration_counter_over_true_bytes": calib, "kernels": kernels}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

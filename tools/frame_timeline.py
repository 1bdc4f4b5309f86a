"""Single-frame pipeline timeline from a rocprofv3 kernel trace: for each
synchronous single-frame run (a run = the dispatches from a head blur to its
k_descriptor), per-kernel duration and the gap before it, median over runs.

    python tools/frame_timeline.py gpurun_out/<dir>/run_kernel_trace.csv [--grid-desc N] [--last K]
"""
import argparse
import csv
import statistics
from collections import defaultdict


def runs(rows):
    out, cur = [], []
    for r in rows:
        if "sift_amd::" not in r["Kernel_Name"]:
            continue
        cur.append(r)
        if "k_descriptor" in r["Kernel_Name"]:
            out.append(cur)
            cur = []
    return out


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("sift_amd::", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--desc", default="k_descriptor<256>", help="descriptor template of the runs to keep")
    ap.add_argument("--first-grid", type=int, default=0, help="keep runs whose first dispatch has this grid x")
    ap.add_argument("--last", type=int, default=30, help="use the last K matching runs")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rs = [r for r in runs(rows) if a.desc in r[-1]["Kernel_Name"]
          and (not a.first_grid or int(r[0]["Grid_Size_X"]) == a.first_grid)]
    sig = defaultdict(list)
    for r in rs:
        sig[tuple((short(x["Kernel_Name"]), x["Grid_Size_X"]) for x in r)].append(r)
    key, group = max(sig.items(), key=lambda kv: len(kv[1]))
    group = group[-a.last:]
    print(f"{len(group)} runs of {len(key)} dispatches")
    tot_k = tot_g = 0.0
    for i, (name, grid) in enumerate(key):
        dur = statistics.median((int(r[i]["End_Timestamp"]) - int(r[i]["Start_Timestamp"])) / 1e3 for r in group)
        gap = statistics.median((int(r[i]["Start_Timestamp"]) - int(r[i - 1]["End_Timestamp"])) / 1e3
                                for r in group) if i else 0.0
        tot_k += dur
        tot_g += gap
        print(f"{i:3d} {name:40s} grid {grid:>9s}  {dur:7.2f} us  gap {gap:6.2f}")
    span = statistics.median((int(r[-1]["End_Timestamp"]) - int(r[0]["Start_Timestamp"])) / 1e3 for r in group)
    print(f"kernels {tot_k:.1f} us + gaps {tot_g:.1f} us; first start -> last end {span:.1f} us")


if __name__ == "__main__":
    main()

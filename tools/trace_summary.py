"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by kernel
name and grid size (= pyramid octave for the per-octave kernels).

    python tools/trace_summary.py gpurun_out/prof_TAG/run_kernel_trace.csv > profiles/<round>/kernel_trace_summary.json
"""
import csv
import json
import sys
from collections import defaultdict


def main(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = [{"kernel": k, "grid_size": g, "launches": len(v), "avg_us": round(sum(v) / len(v), 3),
             "min_us": round(min(v), 3), "total_us": round(sum(v), 1)} for (k, g), v in acc.items()]
    rows.sort(key=lambda r: -r["total_us"])
    json.dump(rows, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Mean kernel durations (us) of single-frame kernel traces, side by side.
    python tools/lat_summary.py DIR1 DIR2 ..."""
import csv
import glob
import sys
from collections import defaultdict

runs = {}
for d in sys.argv[1:]:
    agg = defaultdict(list)
    for f in glob.glob(f"{d}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sift_amd::", "")[:30]
            agg[(n, r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    runs[d] = {k: sum(v) / len(v) for k, v in agg.items() if len(v) >= 20}
keys = sorted(set().union(*runs.values()), key=lambda k: -max(r.get(k, 0) for r in runs.values()))
print(f"{'kernel':32s} {'grid':>8s} " + " ".join(f"{d[-12:]:>12s}" for d in runs))
for k in keys:
    print(f"{k[0]:32s} {k[1]:>8s} " + " ".join(f"{runs[d].get(k, 0):12.2f}" for d in runs))
print(f"{'sum':41s} " + " ".join(f"{sum(runs[d].values()):12.2f}" for d in runs))

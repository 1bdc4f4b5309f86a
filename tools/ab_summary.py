"""Per-kernel mean duration (us) of each tools/ab_prof.sh run, side by side.
    python tools/ab_summary.py NAME1 NAME2 ..."""
import csv
import glob
import sys

runs = {}
for n in sys.argv[1:]:
    g = {}
    for f in glob.glob(f"gpurun_out/abp_{n}/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sift_amd::", "")[:24], r["Grid_Size_X"])
            g.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    runs[n] = {k: (len(v), sum(v) / len(v)) for k, v in g.items() if len(v) >= 10}
keys = sorted(set().union(*[set(r) for r in runs.values()]), key=lambda k: -max(r.get(k, (0, 0))[1] for r in runs.values()))
print(f"{'kernel':26s} {'grid':>8s} " + " ".join(f"{n:>10s}" for n in runs))
tot = {n: 0.0 for n in runs}
for k in keys:
    vals = [runs[n].get(k, (0, 0.0)) for n in runs]
    for n, v in zip(runs, vals):
        tot[n] += v[1]
    print(f"{k[0]:26s} {k[1]:>8s} " + " ".join(f"{v[1]:10.2f}" for v in vals))
print(f"{'sum of means':35s} " + " ".join(f"{tot[n]:10.2f}" for n in runs))

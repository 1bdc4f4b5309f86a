"""Two-stream overlap from a rocprofv3 kernel trace of tools/batch_sweep.py
(--batches 16 --streams 2): per kernel, its mean duration and the fraction of
its time during which a kernel of the other queue was running; and the whole
window's busy union vs the serial sum.
    python tools/overlap_summary.py gpurun_out/DIR"""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(f"{sys.argv[1]}/*kernel_trace.csv"):
    rows += list(csv.DictReader(open(f)))
rows = [r for r in rows if int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) > 4096 or "k_order" in r["Kernel_Name"]]
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
       r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sift_amd::", "")[:28]) for r in rows]
ks.sort()
queues = sorted({k[2] for k in ks})
# skip the first/last 20 % (warmup, tail)
t0 = ks[0][0] + (ks[-1][1] - ks[0][0]) * 0.2
t1 = ks[0][0] + (ks[-1][1] - ks[0][0]) * 0.8
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
byq = defaultdict(list)
for k in win:
    byq[k[2]].append((k[0], k[1]))


def overlap(a0, a1, ivs):
    tot = 0
    for b0, b1 in ivs:
        if b1 <= a0 or b0 >= a1:
            continue
        tot += min(a1, b1) - max(a0, b0)
    return tot


agg = defaultdict(lambda: [0, 0.0, 0.0])
for s, e, q, n in win:
    other = [iv for qq, ivs in byq.items() if qq != q for iv in ivs]
    a = agg[n]
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2] += overlap(s, e, other) / 1e3
print(f"queues {queues}  window {(t1 - t0) / 1e3:.0f} us")
print(f"{'kernel':30s} {'n':>4s} {'mean_us':>8s} {'overlapped':>10s}")
for n, (c, d, o) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{n:30s} {c:4d} {d / c:8.2f} {o / d:10.2f}")
ser = sum(e - s for s, e, q, n in win)
# union of busy time
iv = sorted((s, e) for s, e, q, n in win)
u, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        u += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
u += ce - cs
print(f"serial sum {ser / 1e3:.0f} us, busy union {u / 1e3:.0f} us, window {(t1 - t0) / 1e3:.0f} us")

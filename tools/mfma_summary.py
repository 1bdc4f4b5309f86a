"""Per-dispatch MFMA counters of the matcher kernel from tools/match_pmc.sh.

Usage: python3 tools/mfma_summary.py TAG > profiles/roundN/mfma_counters.json
Reads gpurun_out/mpmc_TAG_p{1,2}/run_counter_collection.csv; averages each
counter over the dispatches of a matcher kernel with the same (name, grid size).

MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (kernel duration x 2.4 GHz x
1024 SIMDs), the duration from the same pass's kernel trace: the fraction of
the chip's matrix-pipe cycles at the peak clock (under load the clock is lower,
so this understates busy a little).  The round-2 figure divided by
GRBM_GUI_ACTIVE / 8 instead; that counter does not track the dispatch's
duration (it read 3.8 GHz-equivalent on the round-3 kernel), so it is kept
only as a raw counter.
"""
import csv
import json
import re
import sys
from collections import defaultdict

KEEP = ["SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT",
        "SQ_ACTIVE_INST_LDS"]


def kname(row):
    """Short kernel name: k_match_single / k_match_direct / k_match_batch ..."""
    m = re.search(r"(k_match\w*)", row["Kernel_Name"])
    return m.group(1) if m else row["Kernel_Name"]


def main(tag):
    vals = defaultdict(lambda: defaultdict(list))  # grid -> counter -> [per dispatch]
    for p in (1, 2):
        per = defaultdict(lambda: defaultdict(float))  # (grid, dispatch) -> counter -> sum over rows
        with open(f"gpurun_out/mpmc_{tag}_p{p}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                if "k_match" not in row["Kernel_Name"] or "prep" in row["Kernel_Name"]:
                    continue
                per[((kname(row), int(row["Grid_Size"])), row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (grid, _), cs in per.items():
            for c, v in cs.items():
                if c in KEEP and not (p == 2 and c == "GRBM_GUI_ACTIVE"):
                    vals[grid][c].append(v)
    dur = defaultdict(list)  # grid -> kernel durations (us) of pass 1
    with open(f"gpurun_out/mpmc_{tag}_p1/run_kernel_trace.csv") as f:
        for row in csv.DictReader(f):
            if "k_match" in row["Kernel_Name"] and "prep" not in row["Kernel_Name"]:
                grid = (kname(row), int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]))
                dur[grid].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    dur_kt = defaultdict(list)  # unprofiled durations (kernel-trace-only run), if present
    try:
        with open(f"gpurun_out/mpmc_{tag}_kt/run_kernel_trace.csv") as f:
            for row in csv.DictReader(f):
                if "k_match" in row["Kernel_Name"] and "prep" not in row["Kernel_Name"]:
                    grid = (kname(row), int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]))
                    dur_kt[grid].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    except FileNotFoundError:
        pass
    out = []
    for grid in sorted(vals):
        d = {"kernel": grid[0], "grid_size": grid[1], "dispatches": len(vals[grid]["SQ_INSTS_MFMA"])}
        for c in KEEP:
            xs = vals[grid][c]
            if xs:
                d[c if c != "GRBM_GUI_ACTIVE" else "GRBM_GUI_ACTIVE_sum_xcd"] = round(sum(xs) / len(xs), 1)
        if dur.get(grid):
            us = sum(dur[grid]) / len(dur[grid])
            d["kernel_us"] = round(us, 3)
            d["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (us * 1e-6 * 2.4e9 * 1024), 4)
        if dur_kt.get(grid):
            ks = sorted(dur_kt[grid])[len(dur_kt[grid]) // 10:]  # first tenth: warm-up
            ukt = sum(ks) / len(ks)
            d["kernel_us_unprofiled"] = round(ukt, 3)
            d["unprofiled_launches"] = len(ks)
            d["mfma_busy_frac_unprofiled"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (ukt * 1e-6 * 2.4e9 * 1024), 4)
            # Both methods side by side: same_pass divides by the
            # --pmc pass's own (counter-stretched) duration; cross_run by a
            # separate kernel-trace run's duration at a nominal 2.4 GHz.  Round 2
            # reported same_pass only; compare rounds on the same method.
            d["mfma_busy_methods"] = {"same_pass": d.get("mfma_busy_frac"), "cross_run_2p4ghz": d["mfma_busy_frac_unprofiled"]}
        out.append(d)
    json.dump({"command": f"tools/match_pmc.sh {tag} (two --pmc passes, kernel trace only, over tools/match_pmc.py); "
                          f"python3 tools/mfma_summary.py {tag}",
               "note": "matcher kernels (int8 MFMA) per dispatch; MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / "
                       "(kernel duration x 2.4 GHz x 1024 SIMDs), the duration from the same --pmc pass's kernel "
                       "trace (stretched by the counters) and, _unprofiled, from a kernel-trace-only run of the "
                       "same workload (400x the calls, first tenth dropped) at a nominal 2.4 GHz -- two runs mixed, so "
                       "mfma_busy_methods lists both; round 2's numbers are same_pass; SQ_VALU_MFMA_BUSY_CYCLES = 32 per MFMA",
               "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Per-dispatch MFMA counters of the matcher kernel from tools/match_pmc.sh.

Usage: python3 tools/mfma_summary.py TAG > profiles/roundN/mfma_counters.json
Reads gpurun_out/mpmc_TAG_p{1,2}/run_counter_collection.csv; averages each
counter over the dispatches of k_match with the same grid size.  MFMA busy
fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs).
"""
import csv
import json
import sys
from collections import defaultdict

KEEP = ["SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_LDS_BANK_CONFLICT",
        "SQ_ACTIVE_INST_LDS"]


def main(tag):
    vals = defaultdict(lambda: defaultdict(list))  # grid -> counter -> [per dispatch]
    for p in (1, 2):
        per = defaultdict(lambda: defaultdict(float))  # (grid, dispatch) -> counter -> sum over rows
        with open(f"gpurun_out/mpmc_{tag}_p{p}/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                if "k_match<" not in row["Kernel_Name"] and not row["Kernel_Name"].endswith("k_match"):
                    if "k_match" not in row["Kernel_Name"] or "prep" in row["Kernel_Name"]:
                        continue
                per[(int(row["Grid_Size"]), row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (grid, _), cs in per.items():
            for c, v in cs.items():
                if c in KEEP and not (p == 2 and c == "GRBM_GUI_ACTIVE"):
                    vals[grid][c].append(v)
    out = []
    for grid in sorted(vals):
        d = {"grid_size": grid, "dispatches": len(vals[grid]["SQ_INSTS_MFMA"])}
        for c in KEEP:
            xs = vals[grid][c]
            if xs:
                d[c if c != "GRBM_GUI_ACTIVE" else "GRBM_GUI_ACTIVE_sum_xcd"] = round(sum(xs) / len(xs), 1)
        g = d.get("GRBM_GUI_ACTIVE_sum_xcd")
        if g:
            d["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 4)
        out.append(d)
    json.dump({"command": f"tools/match_pmc.sh {tag} (two --pmc passes, kernel trace only, over tools/match_pmc.py); "
                          f"python3 tools/mfma_summary.py {tag}",
               "note": "k_match (int8 MFMA) per dispatch; MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / "
                       "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), GRBM_GUI_ACTIVE summed over the 8 XCDs",
               "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Compare bench.py --roofline-only's event-timed k_blur average with the
rocprofv3 kernel-trace of the same command (kernel-only durations).

    python tools/roofline_check.py gpurun_out/roof_TAG.json gpurun_out/roof_TAG/run_kernel_trace.csv
"""
import csv
import json
import sys


def main(bench_json, trace_csv):
    with open(bench_json) as f:
        line = [l for l in f if l.strip().startswith("{")][-1]
    roof = json.loads(line)["roofline"]
    groups = {}
    for r in csv.DictReader(open(trace_csv)):
        if "k_blur" in r["Kernel_Name"]:
            key = (r["Kernel_Name"], r.get("Grid_Size", ""), r.get("Grid_Size_X", ""), r.get("Grid_Size_Y", ""),
                   r.get("Grid_Size_Z", ""))
            groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    # The timed launches (steps x repetitions per (kernel, grid)); the handle's
    # warm-up frames (a few launches per grid, incl. one-frame grids of a
    # batch handle) are left out.
    top = max(len(v) for v in groups.values())
    durs = [d for v in groups.values() if len(v) >= top // 2 for d in v]
    avg = sum(durs) / len(durs)
    out = {"bench_avg_launch_us": roof["avg_launch_us"], "rocprof_avg_us": round(avg, 3), "rocprof_launches": len(durs),
           "ratio_bench_over_rocprof": round(roof["avg_launch_us"] / avg, 3),
           "rocprof_groups_kept": sum(1 for v in groups.values() if len(v) >= top // 2),
           "rocprof_achieved_GBps": round(roof["algo_bytes_per_launch"] / avg / 1e3, 1),
           "note": "bench brackets every launch with HIP events (includes dispatch latency); rocprof counts kernel "
                   "execution only; warm-up launches (fewer per (kernel, grid) than the timed ones) excluded"}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

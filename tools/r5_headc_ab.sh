#!/bin/bash
# Head node A/B: re-pointed every frame vs only when the input changes
# (single-frame latency through Python, alternating builds).
set -o pipefail
: > gpurun_out/headc_ab.jsonl
for lib in base headc base headc; do
  SIFT_HIP_LIB=ab/$lib.so timeout -k 10 120 python3 tools/lat_configs.py --reps 200 >> gpurun_out/headc_ab.jsonl 2> gpurun_out/headc_ab.err || { tail -5 gpurun_out/headc_ab.err; exit 1; }
done
cat gpurun_out/headc_ab.jsonl

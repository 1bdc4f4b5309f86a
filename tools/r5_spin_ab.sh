#!/bin/bash
# Sync wait A/B: hipStreamSynchronize vs polling hipStreamQuery in sync_lanes
# (single-frame latency through Python, alternating builds).
set -o pipefail
: > gpurun_out/spin_ab.jsonl
for lib in base spin base spin; do
  SIFT_HIP_LIB=ab/$lib.so timeout -k 10 120 python3 tools/lat_configs.py --reps 200 >> gpurun_out/spin_ab.jsonl 2> gpurun_out/spin_ab.err || { tail -5 gpurun_out/spin_ab.err; exit 1; }
done
cat gpurun_out/spin_ab.jsonl

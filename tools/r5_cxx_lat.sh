#!/bin/bash
# Synchronous single-frame latency from C++ (detection_example --device: the
# drop-in's detectAndComputeDevice loop) next to the Python surface's
# (tools/lat_configs.py), same box.
set -o pipefail
B=another-cuda-sift_amd/lib/detection_example
: > gpurun_out/cxx_lat.jsonl
for args in "--width 1920 --height 1200 --octaves 3" "--width 752 --height 480" "--width 1920 --height 1200" "--width 1600 --height 900" "--width 1920 --height 1200 --octaves 3"; do
  timeout -k 10 60 $B $args --device --iters 200 2>&1 | grep sync_ms >> gpurun_out/cxx_lat.jsonl || exit 1
done
timeout -k 10 120 python3 tools/lat_configs.py --reps 200 >> gpurun_out/cxx_lat.jsonl 2> gpurun_out/cxx_lat.err || { tail -5 gpurun_out/cxx_lat.err; exit 1; }
cat gpurun_out/cxx_lat.jsonl

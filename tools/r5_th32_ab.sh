#!/bin/bash
# Blur tile height A/B (64-row tiles with 8 / 4 waves vs 32-row tiles with 4
# waves): single-frame latency at the reference configurations and C2
# throughput (16-frame batches on 2 streams), alternating builds.
set -o pipefail
: > gpurun_out/th32_ab.jsonl
for lib in base th32 base th32; do
  SIFT_HIP_LIB=ab/$lib.so timeout -k 10 120 python3 tools/lat_configs.py --reps 40 >> gpurun_out/th32_ab.jsonl 2> gpurun_out/th32_ab.err || { tail -5 gpurun_out/th32_ab.err; exit 1; }
  echo "{\"lib\": \"$lib\", \"sweep\": 1}" >> gpurun_out/th32_ab.jsonl
  SIFT_HIP_LIB=ab/$lib.so timeout -k 10 120 python3 tools/batch_sweep.py --batches 16 --streams 2 --frames 320 >> gpurun_out/th32_ab.jsonl 2>> gpurun_out/th32_ab.err || { tail -5 gpurun_out/th32_ab.err; exit 1; }
done
cat gpurun_out/th32_ab.jsonl

#!/bin/bash
# Sync latency A/B: stream sync vs last-frame event sync (tools/lat_configs.py), interleaved.
set -o pipefail
: > gpurun_out/sync_ab.jsonl
for v in sy0 sy1 sy0 sy1; do
  SIFT_HIP_LIB=ab/$v.so timeout -k 10 120 python tools/lat_configs.py --reps 60 >> gpurun_out/sync_ab.jsonl 2> gpurun_out/sync_ab.err || { tail -5 gpurun_out/sync_ab.err; exit 1; }
done
cat gpurun_out/sync_ab.jsonl

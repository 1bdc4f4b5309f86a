#!/bin/bash
# s_setprio for large windows (orientation, descriptor): single-frame sync latency and batch throughput.
set -o pipefail
: > gpurun_out/prio_ab.jsonl
for v in p0 pO8 pO4 pOD p0 pO8 pO4 pOD; do
  SIFT_HIP_LIB=ab/$v.so timeout -k 10 120 python tools/lat_configs.py --reps 60 >> gpurun_out/prio_ab.jsonl 2> gpurun_out/prio_ab.err || { tail -5 gpurun_out/prio_ab.err; exit 1; }
done
cat gpurun_out/prio_ab.jsonl
AB_BATCH=16 bash tools/ab_run.sh p0 pOD

#!/bin/bash
# Serialized per-kernel durations (rocprofv3 kernel trace over
# tools/profile_frames.py --batch 8) for each ab/NAME.so.
# Usage: tools/ab_prof.sh NAME1 NAME2 ...; summary: tools/ab_summary.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in "$@"; do
  SIFT_HIP_LIB=ab/$N.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/abp_$N -o run --output-format csv -- python3 tools/profile_frames.py --frames 20 --batch ${AB_BATCH:-16} > gpurun_out/abp_$N.log 2>&1 || { echo "$N prof failed"; tail -5 gpurun_out/abp_$N.log; exit 1; }
done
echo prof done

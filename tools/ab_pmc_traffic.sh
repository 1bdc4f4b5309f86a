#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes, kernel trace only) of
# tools/profile_frames.py --batch 16 for each ab/NAME.so; summarise with
# tools/pmc_summary.py NAMEtraffic.  Usage: tools/ab_pmc_traffic.sh NAME1 ...
# PF_ARGS: extra profile_frames.py arguments (e.g. --octaves 1); AB_TAG: a
# suffix for the output directories (NAME${AB_TAG}traffic_p3/4).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for N in "$@"; do
  i=2
  for C in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    SIFT_HIP_LIB=ab/$N.so timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${N}${AB_TAG}traffic_p$i -o run --output-format csv -- python3 tools/profile_frames.py --frames 5 --batch ${AB_BATCH:-16} ${PF_ARGS} > gpurun_out/${N}${AB_TAG}traffic_p$i.log 2>&1 || { echo "$N $C failed"; tail -5 gpurun_out/${N}${AB_TAG}traffic_p$i.log; exit 1; }
  done
done
echo traffic done

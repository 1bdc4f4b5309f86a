#!/bin/bash
# A/B of library builds on the GPU box: interleaved C2 throughput runs
# (tools/batch_sweep.py, batch 8, 2 streams) of each ab/NAME.so.
# Usage: tools/ab_run.sh NAME1 NAME2 ... (after tools/ab_build.sh)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for N in "$@"; do
    SIFT_HIP_LIB=ab/$N.so timeout -k 10 120 python tools/batch_sweep.py --batches ${AB_BATCH:-16} --streams 2 --frames 800 > gpurun_out/ab_$N.$rep.json 2>&1 || { echo "$N failed"; tail -5 gpurun_out/ab_$N.$rep.json; exit 1; }
    echo "$N rep$rep $(tail -1 gpurun_out/ab_$N.$rep.json)"
  done
done

#!/bin/bash
# batch_sweep throughput (16-frame batches, STREAMS streams) for each ab/NAME.so,
# REPS interleaved repetitions.  Usage: tools/r2_sweep.sh "NAME1 NAME2 ..."
set -o pipefail
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-3}); do
  for n in $1; do
    r=$(SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 python3 tools/batch_sweep.py --batches 16 --streams ${STREAMS:-2} --frames 960 2>&1 | tail -1) || { echo "$n failed: $r"; exit 1; }
    echo "$n $r"
  done
done

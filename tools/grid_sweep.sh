#!/bin/bash
# C2 throughput (batch 8, 2 streams) for descriptor / orientation grid sizes
# (SIFT_DESC_WGS / SIFT_ORI_WGS workgroups per frame): co-residency of the
# latency-bound keypoint kernels with the other stream's pyramid kernels.
# Usage: tools/grid_sweep.sh "ENV1" "ENV2" ...  (each a space-free VAR=val[,VAR=val])
set -o pipefail
mkdir -p gpurun_out
run() { echo "$1 $(env ${1//,/ } timeout -k 10 120 python tools/batch_sweep.py --batches 8 --streams 2 --frames 800 | tail -1)"; }
for rep in 1 2; do
  for c in "$@"; do run "$c" || exit 1; done
done

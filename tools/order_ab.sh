#!/bin/bash
# k_order A/B: kernel-trace stats of single frames (tools/profile_frames.py,
# batch 1 and batch 16) for the default build and ab/ord0.so.
set -o pipefail
TAG=${1:-ord}
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in default ord0; do
  if [ $V = default ]; then LIBENV=""; else LIBENV="ab/$V.so"; fi
  for B in 1 16; do
    SIFT_HIP_LIB=$LIBENV timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${V}_b$B -o run --output-format csv -- python3 tools/profile_frames.py --frames 20 --batch $B > gpurun_out/${TAG}_${V}_b$B.log 2>&1 || { echo "$V b$B failed"; exit 1; }
  done
done
echo done

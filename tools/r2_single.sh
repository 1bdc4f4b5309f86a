#!/bin/bash
# Single-frame (drop-in path) kernel trace + eager stage table.  Usage: tools/r2_single.sh TAG
set -o pipefail
TAG=${1:-s}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/single_$TAG -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/single_$TAG.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/single_$TAG.log; exit 1; }
timeout -k 10 120 python3 tools/profile_frames.py --frames 30 --eager > gpurun_out/single_eager_$TAG.log 2>&1 || { echo "eager failed"; tail -5 gpurun_out/single_eager_$TAG.log; exit 1; }
cat gpurun_out/single_eager_$TAG.log

#!/bin/bash
# Single-frame per-kernel timelines (C2 and 752x480 auto octaves): kernel
# trace of synchronous single frames, summarised by tools/frame_timeline.py.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-tl}
# LIB=ab/X.so: an A/B build instead of the tree's library
[ -n "$LIB" ] && export SIFT_HIP_LIB=$LIB
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_c2 -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/${TAG}_c2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_752 -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 --width 752 --height 480 --octaves 0 > gpurun_out/${TAG}_752.log 2>&1 || exit 1
python3 tools/frame_timeline.py gpurun_out/${TAG}_c2/run_kernel_trace.csv --last 20 > gpurun_out/${TAG}_c2.txt
python3 tools/frame_timeline.py gpurun_out/${TAG}_752/run_kernel_trace.csv --last 20 > gpurun_out/${TAG}_752.txt
cat gpurun_out/${TAG}_c2.txt gpurun_out/${TAG}_752.txt

#!/bin/bash
# Kernel + memory-copy traces of the 3-lane host pipeline: device frames (dev 1)
# vs pinned host frames moved by DMA (dev 3) and read zero-copy (dev 2).
set -o pipefail
export TMPDIR=/tmp
for m in 1 3 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/hpt_$m -o run --output-format csv -- another-cuda-sift_amd/lib/host_pipeline_bench 3 6 60 2 $m > gpurun_out/hpt_$m.log 2>&1 || { tail -5 gpurun_out/hpt_$m.log; exit 1; }
done
ls gpurun_out/hpt_1 gpurun_out/hpt_3

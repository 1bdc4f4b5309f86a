#!/bin/bash
# Host input modes of tools/host_pipeline_bench.cpp (3 lanes x 6 frames, no
# result copies): device frames, pinned zero-copy, DMA, and the two DMA
# diagnostics (cross-stream wait alone, unordered DMA).
set -o pipefail
: > gpurun_out/host_modes.jsonl
for args in "3 6 300 2 1" "3 6 300 2 4" "3 6 300 2 5" "3 6 300 2 3" "3 6 300 2 2" "3 6 300 2 0" "1 2 150 2 1" "1 2 150 2 3" "1 2 150 2 2"; do
  timeout -k 10 120 another-cuda-sift_amd/lib/host_pipeline_bench $args >> gpurun_out/host_modes.jsonl 2> gpurun_out/host_modes.err || { tail -5 gpurun_out/host_modes.err; exit 1; }
done
cat gpurun_out/host_modes.jsonl

#!/bin/bash
# Host micro-batched frames: lanes x group size x in-flight sweep (C++ loop, views / copyToHost).
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/host_lanes.jsonl
for args in "3 12 300 3 0 4" "4 16 300 3 0 4" "4 16 300 1 0 4" "4 8 300 3 0 2" "2 8 300 3 0 4" "3 24 300 3 0 8" "4 16 300 2 0 4" "3 12 300 3 0 4"; do
  timeout -k 10 120 $B $args >> gpurun_out/host_lanes.jsonl 2> gpurun_out/host_lanes.err || { tail -5 gpurun_out/host_lanes.err; exit 1; }
done
grep dev gpurun_out/host_lanes.jsonl

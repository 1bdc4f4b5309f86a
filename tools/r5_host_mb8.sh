#!/bin/bash
# Host micro-batched frames with larger groups (C++ loop): group size x in-flight x read-back mode.
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/host_mb8.jsonl
for args in "3 24 300 3 0 8" "3 24 300 1 0 8" "3 32 300 3 0 8" "3 16 300 3 0 8" "2 16 300 3 0 8" "3 36 300 3 0 12" "3 24 300 3 0 6" "3 24 300 2 0 8" "3 24 300 3 0 8" "3 24 300 1 0 8" "3 24 300 3 1 8"; do
  timeout -k 10 120 $B $args >> gpurun_out/host_mb8.jsonl 2> gpurun_out/host_mb8.err || { tail -5 gpurun_out/host_mb8.err; exit 1; }
done
grep dev gpurun_out/host_mb8.jsonl

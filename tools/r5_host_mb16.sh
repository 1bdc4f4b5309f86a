#!/bin/bash
# Host and device micro-batched frames at 8 / 12 / 16-frame groups (C++ loop, views).
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/host_mb16.jsonl
for args in "3 24 400 3 0 8" "3 48 400 3 0 16" "3 32 400 3 0 16" "2 32 400 3 0 16" "3 36 400 3 0 12" "3 24 400 3 1 8" "3 48 400 3 1 16" "3 24 400 3 0 8"; do
  timeout -k 10 120 $B $args >> gpurun_out/host_mb16.jsonl 2> gpurun_out/host_mb16.err || { tail -5 gpurun_out/host_mb16.err; exit 1; }
done
grep dev gpurun_out/host_mb16.jsonl

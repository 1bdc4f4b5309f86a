#!/bin/bash
# Micro-batched host frames: per-submit time distribution by descriptor read-back mode.
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/mbh_diag.jsonl
for args in "3 12 300 2 0 4" "3 12 300 0 0 4" "3 12 300 1 0 4" "3 6 300 1 0 1" "2 8 300 1 0 4" "3 12 300 1 0 2"; do
  timeout -k 10 120 $B $args >> gpurun_out/mbh_diag.jsonl 2> gpurun_out/mbh_diag.err || { tail -5 gpurun_out/mbh_diag.err; exit 1; }
done
grep dev gpurun_out/mbh_diag.jsonl

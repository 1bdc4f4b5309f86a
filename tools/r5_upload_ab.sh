#!/bin/bash
# Host-input upload A/B (tools/host_pipeline_bench, 3 lanes x 6 frames, no
# result copies): hardware queues 4 vs 8 for the copy-stream modes, and the
# lane-stream DMA upload build (ab/L_uplane, -DSIFT_AB_UPLOAD_LANE) vs the
# zero-copy read (ab/L_upl0) for submit().
set -o pipefail
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/upload_ab.jsonl
run() { echo "{\"tag\": \"$1\"}" >> gpurun_out/upload_ab.jsonl; shift; timeout -k 10 120 "$@" >> gpurun_out/upload_ab.jsonl 2> gpurun_out/upload_ab.err || { tail -5 gpurun_out/upload_ab.err; exit 1; }; }
run hwq4 $B 3 6 300 2 4
run hwq8 env GPU_MAX_HW_QUEUES=8 $B 3 6 300 2 4
run hwq8 env GPU_MAX_HW_QUEUES=8 $B 3 6 300 2 5
run hwq8 env GPU_MAX_HW_QUEUES=8 $B 3 6 300 2 3
run hwq8 env GPU_MAX_HW_QUEUES=8 $B 3 6 300 2 0
run hwq8 env GPU_MAX_HW_QUEUES=8 $B 3 6 300 2 1
run upl0 env LD_LIBRARY_PATH=ab/L_upl0 $B 3 6 300 2 0
run uplane env LD_LIBRARY_PATH=ab/L_uplane $B 3 6 300 2 0
run uplane env LD_LIBRARY_PATH=ab/L_uplane $B 3 6 300 1 0
run uplane env LD_LIBRARY_PATH=ab/L_uplane $B 1 2 150 2 0
run upl0 env LD_LIBRARY_PATH=ab/L_upl0 $B 1 2 150 2 0
run uplane_hwq8 env GPU_MAX_HW_QUEUES=8 LD_LIBRARY_PATH=ab/L_uplane $B 3 6 300 2 0
cat gpurun_out/upload_ab.jsonl

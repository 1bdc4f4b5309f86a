#!/bin/bash
# Round-5 host/lanes measurements: device submit/wait at 4 vs 8 hardware
# queues per process, the C++ host pipeline (per-call wall times), and both
# descriptor modes (throughput + sync latency).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/dev_pipeline_time.py > gpurun_out/hwq_ab.jsonl 2> gpurun_out/hwq_ab.err || { tail -5 gpurun_out/hwq_ab.err; exit 1; }
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python tools/dev_pipeline_time.py >> gpurun_out/hwq_ab.jsonl 2>> gpurun_out/hwq_ab.err || { tail -5 gpurun_out/hwq_ab.err; exit 1; }
: > gpurun_out/host_pipeline.jsonl
for args in "3 6 200 1 0" "3 6 200 0 0" "3 6 200 2 0" "3 6 200 2 1" "1 1 100 1 0"; do
  timeout -k 10 120 another-cuda-sift_amd/lib/host_pipeline_bench $args >> gpurun_out/host_pipeline.jsonl 2> gpurun_out/host_pipeline.err || { tail -5 gpurun_out/host_pipeline.err; exit 1; }
done
timeout -k 10 300 python tools/desc_mode_bench.py > gpurun_out/desc_mode.jsonl 2> gpurun_out/desc_mode.err || { tail -5 gpurun_out/desc_mode.err; exit 1; }
cat gpurun_out/hwq_ab.jsonl gpurun_out/host_pipeline.jsonl gpurun_out/desc_mode.jsonl

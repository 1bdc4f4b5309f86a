#!/bin/bash
# Micro-batched device submits: GPU tests, then submit/wait throughput over
# (lanes, depth, micro-batch).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mb_lanes.log 2>&1
rc=$?; echo "lanes tests rc=$rc"; tail -3 gpurun_out/pytest_mb_lanes.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mb.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_mb.log; [ $rc -eq 0 ] || exit 1
DEV_CONFIGS="3:6:1,2:8:4,2:12:4,3:12:4,2:6:3,3:9:3,2:8:2,3:6:2,4:16:4" timeout -k 10 300 python tools/dev_pipeline_time.py > gpurun_out/mb_dev.jsonl 2> gpurun_out/mb_dev.err || { tail -5 gpurun_out/mb_dev.err; exit 1; }
cat gpurun_out/mb_dev.jsonl

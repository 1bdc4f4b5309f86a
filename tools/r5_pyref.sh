#!/bin/bash
# Python result refresh change: every GPU test, then the synchronous latency through Python.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/pyref_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pyref_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 tools/lat_configs.py --reps 200 > gpurun_out/pyref_lat.jsonl 2> gpurun_out/pyref_lat.err || { tail -5 gpurun_out/pyref_lat.err; exit 1; }
timeout -k 10 60 another-cuda-sift_amd/lib/detection_example --width 1920 --height 1200 --octaves 3 --device --iters 200 | grep sync_ms >> gpurun_out/pyref_lat.jsonl
cat gpurun_out/pyref_lat.jsonl

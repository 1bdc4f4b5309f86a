#!/bin/bash
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_match_sidecar.py tests/test_gpu_input.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mbh2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_mbh2.log; [ $rc -eq 0 ] || exit 1
bash tools/r5_bench_quick.sh

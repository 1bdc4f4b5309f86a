#!/bin/bash
# Detector-owned host results (sift_hip_results_host): parity tests, then the
# pipelined host loop with views vs copyToHost (C++ tool and bench legs).
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lanes.py > gpurun_out/views_pytest.log 2>&1 || { tail -30 gpurun_out/views_pytest.log; exit 1; }
tail -3 gpurun_out/views_pytest.log
B=another-cuda-sift_amd/lib/host_pipeline_bench
: > gpurun_out/views_host.jsonl
for args in "3 12 300 3 0 4" "3 12 300 1 0 4" "3 12 300 3 0 4" "3 12 300 1 0 4" "3 6 300 3 0 1" "3 12 300 2 0 4"; do
  timeout -k 10 120 $B $args >> gpurun_out/views_host.jsonl 2> gpurun_out/views_host.err || { tail -5 gpurun_out/views_host.err; exit 1; }
done
grep dev gpurun_out/views_host.jsonl
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_views.json 2> gpurun_out/bench_views.err || { tail -5 gpurun_out/bench_views.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_views.json').read().strip().splitlines()[-1])
print(d['value'], d['sync_ms_per_frame'], json.dumps(d['host_input']))"

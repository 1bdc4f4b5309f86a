#!/bin/bash
# Micro-batched host frames + small-grid copies: GPU tests, the C++ host
# pipeline over (lanes, depth, micro-batch), a short bench run.
set -o pipefail
export TMPDIR=/tmp
B=another-cuda-sift_amd/lib/host_pipeline_bench
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_match_sidecar.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mbh_lanes.log 2>&1
rc=$?; echo "lanes tests rc=$rc"; tail -3 gpurun_out/pytest_mbh_lanes.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_mbh.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_mbh.log; [ $rc -eq 0 ] || exit 1
: > gpurun_out/mbh_modes.jsonl
run() { timeout -k 10 120 "$@" >> gpurun_out/mbh_modes.jsonl 2> gpurun_out/mbh_modes.err || { tail -5 gpurun_out/mbh_modes.err; exit 1; }; }
run $B 3 6 300 1 0 1
run $B 3 12 300 1 0 4
run $B 3 12 300 2 0 4
run $B 2 8 300 1 0 4
run $B 3 12 300 2 1 4
grep dev gpurun_out/mbh_modes.jsonl
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_mbh.json 2> gpurun_out/bench_mbh.err || { tail -5 gpurun_out/bench_mbh.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_mbh.json').read().strip().splitlines()[-1])
print(d['value'], d['sync_ms_per_frame'], json.dumps(d['host_input']), json.dumps(d['device_submit']))"

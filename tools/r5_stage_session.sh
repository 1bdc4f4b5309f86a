#!/bin/bash
# Host frames staged to device memory by a small-grid copy kernel: GPU tests,
# the C++ host pipeline and a short bench run.
set -o pipefail
export TMPDIR=/tmp
B=another-cuda-sift_amd/lib/host_pipeline_bench
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_stage.log; [ $rc -eq 0 ] || exit 1
: > gpurun_out/stage_modes.jsonl
run() { timeout -k 10 120 "$@" >> gpurun_out/stage_modes.jsonl 2> gpurun_out/stage_modes.err || { tail -5 gpurun_out/stage_modes.err; exit 1; }; }
run $B 3 6 300 2 0
run $B 3 6 300 1 0
run $B 3 6 300 0 0
run $B 2 4 300 1 0
run $B 1 2 150 1 0
run $B 1 1 150 1 0
run $B 3 6 300 2 1
grep dev gpurun_out/stage_modes.jsonl
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_stage.json 2> gpurun_out/bench_stage.err || { tail -5 gpurun_out/bench_stage.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_stage.json').read().strip().splitlines()[-1])
print(d['value'], d['sync_ms_per_frame'], json.dumps(d['host_input']), json.dumps(d['device_submit']))"
# copy pool 3 vs 7 workers (staging copy + descriptor read-back), C++ loop
for v in cw3 cw7 cw3 cw7; do
  echo "{\"tag\": \"$v\"}" >> gpurun_out/stage_modes.jsonl
  LD_LIBRARY_PATH=ab/L_$v timeout -k 10 120 $B 3 6 300 1 0 >> gpurun_out/stage_modes.jsonl 2>> gpurun_out/stage_modes.err || exit 1
done
grep -A1 tag gpurun_out/stage_modes.jsonl | grep -v nOct

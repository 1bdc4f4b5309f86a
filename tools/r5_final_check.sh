#!/bin/bash
# Final round-5 check on HEAD: every GPU test, smoke, the default bench command.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 240 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_final.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.txt 2>&1 || { tail -5 gpurun_out/smoke_final.txt; exit 1; }
tail -1 gpurun_out/smoke_final.txt
timeout -k 10 500 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -5 gpurun_out/bench_final.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['sync_ms_per_frame'], d['host_input'].get('pipelined_u8_micro_batch'), d['device_submit'].get('micro_batch',{}).get('f32'))"

#!/bin/bash
# The driver's default bench command, timed.
set -o pipefail
s=$(date +%s)
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
echo "bench seconds: $(( $(date +%s) - s ))"
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['frac'], d['sync_ms_per_frame'], json.dumps(d['host_input'])[:400], json.dumps(d['device_submit'])[:300])"

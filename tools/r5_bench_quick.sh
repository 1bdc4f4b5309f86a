#!/bin/bash
# Short bench run (no CPU baseline) with the host/device pipelined legs.
set -o pipefail
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -5 gpurun_out/bench_quick.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_quick.json').read().strip().splitlines()[-1])
print(d['value'], d['sync_ms_per_frame'], json.dumps(d['host_input']), json.dumps(d['device_submit']))"

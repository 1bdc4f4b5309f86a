#!/bin/bash
# bench.py headline leg: 2 vs 3 streams (16-frame batches) and 3 x 24, interleaved.
set -o pipefail
: > gpurun_out/streams_ab.txt
for rep in 1 2; do
  for cfg in "--streams 2 --batch 16" "--streams 3 --batch 16" "--streams 3 --batch 24"; do
    timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline $cfg > gpurun_out/sab.json 2> gpurun_out/sab.err || { tail -5 gpurun_out/sab.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/sab.json').read().strip().splitlines()[-1])
print('$cfg', d['value'], d['ms_per_frame'], d['roofline']['frac'])" >> gpurun_out/streams_ab.txt
  done
done
cat gpurun_out/streams_ab.txt

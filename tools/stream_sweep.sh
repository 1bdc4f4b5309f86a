#!/bin/bash
# Bench throughput over (streams, batch) pairs.  Usage: bash tools/stream_sweep.sh ["S B" ...]
set -o pipefail
mkdir -p gpurun_out
[ $# -gt 0 ] || set -- "2 16" "3 16" "4 16" "3 8" "4 8" "2 16"
for cfg in "$@"; do
  read s b <<< "$cfg"
  timeout -k 10 200 python bench.py --streams $s --batch $b --no-cpu-baseline > gpurun_out/ss_${s}_$b.json 2>gpurun_out/ss_${s}_$b.err || { echo "fail $cfg"; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ss_${s}_$b.json')); print('streams $s batch $b', d['value'], d['ms_per_frame'])"
done

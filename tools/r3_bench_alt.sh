#!/bin/bash
# Alternating bench lines of ab/NAME.so builds (box-to-box noise is larger than
# most A/B differences; alternate on one box): tools/r3_bench_alt.sh REPS NAME...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
REPS=$1; shift
for r in $(seq 1 $REPS); do
  for n in "$@"; do
    SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/balt_${n}_$r.json 2> gpurun_out/balt_${n}_$r.err || { echo "bench $n failed"; tail -5 gpurun_out/balt_${n}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/balt_${n}_$r.json')); print('$n', $r, d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'c5', d['c5_allgather_match']['batched_match_ms'])"
  done
done

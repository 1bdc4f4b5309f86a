#!/bin/bash
# Single-frame A/B: matcher tests + sweep on the default build, then per
# ab/NAME.so a single-frame kernel trace (30 frames) and the bench's sync latency.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_sab.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_sab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/match_sweep.py 60 > gpurun_out/match_sweep_sab.json 2> gpurun_out/match_sweep_sab.err || { echo "match sweep failed"; exit 1; }
grep -o '"pairs_not_exact": [0-9]*' gpurun_out/match_sweep_sab.json
for n in "$@"; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/sab_$n -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/sab_$n.log 2>&1 || { echo "$n trace failed"; exit 1; }
  python3 tools/trace_summary.py gpurun_out/sab_$n/run_kernel_trace.csv | python3 -c "
import json,sys
rows=json.load(sys.stdin)
tot=sum(r['total_us'] for r in rows if 'rocclr' not in r['kernel'])/30
print('$n kernel us/frame', round(tot,1))
for r in sorted(rows, key=lambda r:-r['total_us'])[:5]: print('   ', r['kernel'][:36], r['grid_size'], r['launches'], r['avg_us'])"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_sab_$n.json 2> gpurun_out/bench_sab_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_sab_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_sab_$n.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'serial', d['single_stream']['ms_per_frame'])"
done

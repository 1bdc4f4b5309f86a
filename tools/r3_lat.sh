#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in $1; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/lat_$2_$n -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/lat_$2_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/lat_$2_$n.log; exit 1; }
  python3 tools/trace_summary.py gpurun_out/lat_$2_$n/run_kernel_trace.csv > gpurun_out/lat_$2_$n.json
  python3 -c "
import json; rows=json.load(open('gpurun_out/lat_$2_$n.json'))
tot=sum(r['total_us'] for r in rows if 'rocclr' not in r['kernel'])/30
blur=sum(r['total_us'] for r in rows if 'blur' in r['kernel'])/30
print('$n kernel us/frame', round(tot,1), 'blur', round(blur,1))
for r in sorted(rows, key=lambda r:-r['total_us'])[:12]: print('   ', r['kernel'][:36], r['grid_size'], r['launches'], r['avg_us'])"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_$2_$n.json 2> gpurun_out/bench_$2_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_$2_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_$2_$n.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'serial', d['single_stream']['ms_per_frame'])"
done

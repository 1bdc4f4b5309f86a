#!/bin/bash
# Extrema A/B: serialized 16-frame and single-frame kernel traces of each
# ab/NAME.so (tools/ab_prof.sh), then the bench line of each.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
NAMES="$*"
AB_BATCH=16 bash tools/ab_prof.sh $NAMES || exit 1
python3 tools/ab_summary.py $NAMES | grep -E "kernel|extrema|sum of"
for n in $NAMES; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/abs_$n -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/abs_$n.log 2>&1 || { echo "$n single failed"; exit 1; }
  python3 tools/trace_summary.py gpurun_out/abs_$n/run_kernel_trace.csv | python3 -c "
import json,sys
for k in json.load(sys.stdin):
    if 'extrema' in k['kernel']: print('  single $n', k['kernel'][:30], k['grid_size'], k['launches'], k['avg_us'], k['min_us'])"
done
for n in $NAMES; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_ex_$n.json 2> gpurun_out/bench_ex_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_ex_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_ex_$n.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'ex', d['stage_us_per_frame_eager'].get('extrema'))"
done

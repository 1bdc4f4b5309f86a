#!/bin/bash
# Blur A/B: the -m gpu suite on the default build, then per ab/NAME.so a
# serialised kernel trace of 16-frame batches (tools/profile_frames.py) and a
# bench line.  Usage: tools/r3_blur_ab.sh TAG "NAME1 ..." [skip-tests]
set -o pipefail
TAG=$1; NAMES=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$3" != skip-tests ]; then
  timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for n in $NAMES; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/bab_${TAG}_$n -o run --output-format csv -- python3 tools/profile_frames.py --frames 20 --batch 16 > gpurun_out/bab_${TAG}_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/bab_${TAG}_$n.log; exit 1; }
  python3 tools/trace_summary.py gpurun_out/bab_${TAG}_$n/run_kernel_trace.csv | python3 -c "
import json,sys
rows=json.load(sys.stdin); tot=0
for k in rows:
    if 'blur' in k['kernel']:
        tot+=k['total_us']/ (20 if True else 1)
        print('  $n', k['kernel'][:40], 'grid', k['grid_size'], 'n', k['launches'], 'avg', k['avg_us'])
print('  $n blur total per batch', round(tot,1))"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_${TAG}_$n.json 2> gpurun_out/bench_${TAG}_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$n.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'serial', d['single_stream']['ms_per_frame'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_us'], 'c5', d['c5_allgather_match']['batched_match_ms'], 'c3', d['match_2k']['ms'])"
done
echo done

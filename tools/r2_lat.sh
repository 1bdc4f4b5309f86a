#!/bin/bash
# GPU tests (default build), then single-frame kernel traces and bench lines
# of each ab/NAME.so.  Usage: tools/r2_lat.sh TAG "NAME1 NAME2 ..." [skip-tests]
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
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/lat_${TAG}_$n -o run --output-format csv -- python3 tools/profile_frames.py --frames 30 > gpurun_out/lat_${TAG}_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/lat_${TAG}_$n.log; exit 1; }
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_${TAG}_$n.json 2> gpurun_out/bench_${TAG}_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_${TAG}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$n.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'serial', d['single_stream']['ms_per_frame'], d['roofline']['frac'])"
done

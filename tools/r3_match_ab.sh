#!/bin/bash
# Matcher A/B: GPU matcher tests (default build), then per ab/NAME.so the
# event-timed C3 / C5 figures (tools/match_time.py) and a kernel trace of the
# matcher workload (tools/match_pmc.py).  Usage: tools/r3_match_ab.sh TAG "NAME1 ..." [skip-tests]
set -o pipefail
TAG=$1; NAMES=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$3" != skip-tests ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -x -k "match or Match" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for n in $NAMES; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 python3 tools/match_time.py > gpurun_out/mt_${TAG}_$n.json 2>&1 || { echo "time $n failed"; tail -5 gpurun_out/mt_${TAG}_$n.json; exit 1; }
  echo "$n $(cat gpurun_out/mt_${TAG}_$n.json)"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/mab_${TAG}_$n -o run --output-format csv -- python3 tools/match_pmc.py > gpurun_out/mab_${TAG}_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/mab_${TAG}_$n.log; exit 1; }
  python3 tools/trace_summary.py gpurun_out/mab_${TAG}_$n/run_kernel_trace.csv | python3 -c "
import json,sys
for k in json.load(sys.stdin):
    if 'match' in k['kernel']: print('  $n', k['kernel'][:34], 'grid', k['grid_size'], 'n', k['launches'], 'avg', k['avg_us'], 'min', k['min_us'])"
done
echo done

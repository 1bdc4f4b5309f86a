#!/bin/bash
# Batched-matcher workgroup shape A/B: per ab/NAME.so the matcher GPU tests,
# event-timed C3/C5 (tools/match_time.py) and a kernel trace of 2000 C5 calls.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
for n in "$@"; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "match or Match" --timeout 120 --timeout-method thread > gpurun_out/pytest_q_$n.log 2>&1; rc=$?; echo "$n $(tail -1 gpurun_out/pytest_q_$n.log)"; [ $rc -eq 0 ] || exit $rc
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 python3 tools/match_time.py > gpurun_out/mt_q_$n.json 2>&1 || { echo "$n failed"; tail -5 gpurun_out/mt_q_$n.json; exit 1; }
  echo "$n $(tail -1 gpurun_out/mt_q_$n.json)"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/q_$n -o run --output-format csv -- python3 tools/match_pmc.py 400 > gpurun_out/q_$n.log 2>&1 || { echo "trace $n failed"; exit 1; }
  python3 - <<PY
import csv, statistics
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in csv.DictReader(open('gpurun_out/q_$n/run_kernel_trace.csv')) if 'k_match_batch' in r['Kernel_Name']]
print('  $n k_match_batch', len(d), 'first200', round(statistics.mean(d[:200]), 2), 'last500', round(statistics.mean(d[-500:]), 2), 'min', min(d))
PY
done

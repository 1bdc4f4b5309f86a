#!/bin/bash
# Single-pair matcher check: matcher GPU tests + 60-pair sweep on the default
# build, then C3 / C5 event timings and a kernel trace of each ab/NAME.so.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "match or Match" --timeout 120 --timeout-method thread > gpurun_out/pytest_c3.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/match_sweep.py 60 > gpurun_out/match_sweep_c3.json 2> gpurun_out/match_sweep_c3.err || { echo "match sweep failed"; tail -5 gpurun_out/match_sweep_c3.err; exit 1; }
grep -o '"pairs_not_exact": [0-9]*' gpurun_out/match_sweep_c3.json
for n in "$@"; do
  for rep in 1 2; do
    SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 python3 tools/match_time.py > gpurun_out/mt_c3d_$n.json 2>&1 || { echo "$n failed"; tail -5 gpurun_out/mt_c3d_$n.json; exit 1; }
    echo "$n $(tail -1 gpurun_out/mt_c3d_$n.json)"
  done
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/c3d_$n -o run --output-format csv -- python3 tools/match_pmc.py 20 > gpurun_out/c3d_$n.log 2>&1 || { echo "trace $n failed"; exit 1; }
  python3 tools/trace_summary.py gpurun_out/c3d_$n/run_kernel_trace.csv | python3 -c "
import json,sys
for k in json.load(sys.stdin):
    if 'match' in k['kernel']: print('  $n', k['kernel'][:34], 'grid', k['grid_size'], 'n', k['launches'], 'avg', k['avg_us'], 'min', k['min_us'])"
done

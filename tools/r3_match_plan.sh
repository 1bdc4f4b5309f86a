#!/bin/bash
# Matcher check on the box: the -m gpu matcher tests and the 60-pair sweep on
# the default build, the per-workgroup timeline of a stamped copy
# (tools/match_wgstamps.py build wgs2) with a kernel trace of the same run, and
# the event-timed C3 / C5 figures (tools/match_time.py).
set -o pipefail
TAG=${1:-m}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "match or Match" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/match_sweep.py 60 > gpurun_out/match_sweep_$TAG.json 2> gpurun_out/match_sweep_$TAG.err || { echo "match sweep failed"; tail -5 gpurun_out/match_sweep_$TAG.err; exit 1; }
tail -c 300 gpurun_out/match_sweep_$TAG.json; echo
SIFT_HIP_LIB=ab/wgs2.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/wgs_$TAG -o run --output-format csv -- python3 tools/match_wgstamps.py run > gpurun_out/wgs_$TAG.json 2> gpurun_out/wgs_$TAG.err || { tail -3 gpurun_out/wgs_$TAG.err; exit 1; }
cat gpurun_out/wgs_$TAG.json
python3 tools/trace_summary.py gpurun_out/wgs_$TAG/run_kernel_trace.csv > gpurun_out/wgs_${TAG}_trace.json && head -16 gpurun_out/wgs_${TAG}_trace.json
timeout -k 10 120 python3 tools/match_time.py > gpurun_out/mt_$TAG.json 2>&1 || { tail -5 gpurun_out/mt_$TAG.json; exit 1; }
cat gpurun_out/mt_$TAG.json

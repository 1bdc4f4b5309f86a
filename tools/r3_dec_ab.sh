#!/bin/bash
# Producer-side decimation A/B: full GPU suite on the default build, then
# serialized 16-frame kernel traces, single-frame traces and bench lines of
# each ab/NAME.so.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_dec.log; [ $rc -eq 0 ] || exit $rc
AB_BATCH=16 bash tools/ab_prof.sh "$@" || exit 1
python3 tools/ab_summary.py "$@" | grep -E "kernel|blur|sum of"
bash tools/r3_lat.sh "$*" dec

#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats.  Usage: tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
# A fault, abort or time limit ends the session (no further GPU step).
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "prof rc=$?"
# Roofline pass alone under rocprofv3: its k_blur average must match bench.py's avg_launch_us.
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/roof_$TAG -o run --output-format csv -- python bench.py --roofline-only --steps 100 > gpurun_out/roof_$TAG.json 2> gpurun_out/roof_$TAG.err
echo "roofline prof rc=$?"

#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_s3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_s3.log
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/match_pmc.sh s3 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/bench_s3.json 2> gpurun_out/bench_s3.err || { echo "bench failed"; tail -20 gpurun_out/bench_s3.err; exit 1; }
cat gpurun_out/bench_s3.json

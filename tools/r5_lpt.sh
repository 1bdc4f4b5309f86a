#!/bin/bash
# Round 5: full GPU suite, bench, single-frame timelines, and the longest-first
# descriptor order A/B (ab/prelpt.so vs ab/lpt.so: batch kernel durations and
# single-frame latency).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_r5f.log 2>&1; rc=$?
echo pytest rc=$rc; tail -4 gpurun_out/pytest_r5f.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_r5f.json 2> gpurun_out/bench_r5f.err; echo bench rc=$?
bash tools/r5_timeline.sh tl5 || exit 1
tools/ab_prof.sh prelpt lpt || exit 1
python3 tools/ab_summary.py prelpt lpt | head -14
for L in prelpt lpt prelpt lpt; do SIFT_HIP_LIB=ab/$L.so timeout -k 10 120 python3 tools/lat_configs.py --reps 40 || exit 1; done

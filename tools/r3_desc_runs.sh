#!/bin/bash
# Descriptor run-accumulator A/B: -m gpu suite on the working-tree build, then
# interleaved throughput and serialized kernel durations of ab/{base,runs,runs5}.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_dr.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dr.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_run.sh base runs runs5 || exit 1
bash tools/ab_prof.sh base runs runs5 || exit 1
python3 tools/ab_summary.py base runs runs5 > gpurun_out/ab_summary_dr.txt 2>&1; tail -30 gpurun_out/ab_summary_dr.txt
echo done

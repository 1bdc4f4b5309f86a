#!/bin/bash
# Round-2 GPU session: parity tests, bench, serialized per-kernel A/B of
# kernel variants (tools/ab_prof.sh), matcher timings.  Usage: tools/r2_session.sh TAG "VARIANTS"
set -o pipefail
TAG=${1:-s1}
VARIANTS=${2:-}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python tools/match_time.py 2000 > gpurun_out/match_$TAG.json 2>&1 || { echo "match_time failed"; tail -5 gpurun_out/match_$TAG.json; exit 1; }
cat gpurun_out/match_$TAG.json
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ -n "$VARIANTS" ]; then
  AB_BATCH=16 bash tools/ab_prof.sh $VARIANTS || exit 1
  python3 tools/ab_summary.py $VARIANTS > gpurun_out/ab_$TAG.txt
  cat gpurun_out/ab_$TAG.txt
fi

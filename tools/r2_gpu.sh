#!/bin/bash
# Round-2 GPU check: -m gpu suite, default bench line, rocprof kernel stats of
# a short bench run.  Usage: tools/r2_gpu.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-g1}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$2" != skip-tests ]; then
  timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/prof_$TAG.log; exit 1; }
echo done

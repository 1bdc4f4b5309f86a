#!/bin/bash
# Round-3 GPU check: test_gpu_parity.py alone (load-order isolation), the whole
# -m gpu suite, the default bench line.  Usage: tools/r3_gpu.sh TAG [skip-tests|only-tests]
set -o pipefail
TAG=${1:-g1}
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/descriptor_exact.txt
if [ "$2" != skip-tests ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_alone_$TAG.log 2>&1
  rc=$?; echo "parity-alone rc=$rc"; tail -4 gpurun_out/pytest_alone_$TAG.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/descriptor_exact.txt gpurun_out/descriptor_exact_$TAG.txt 2>/dev/null
fi
[ "$2" = only-tests ] && exit 0
timeout -k 10 500 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
echo done

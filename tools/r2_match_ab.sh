#!/bin/bash
# GPU tests (default build), then per ab/NAME.so: a kernel trace of the matcher
# workload (tools/match_pmc.py: C3 single pairs + the C5 batched call) and the
# bench line's match figures.  Usage: tools/r2_match_ab.sh TAG "NAME1 ..." [skip-tests]
set -o pipefail
TAG=$1; NAMES=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$3" != skip-tests ]; then
  timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || exit $rc
fi
for n in $NAMES; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/mab_${TAG}_$n -o run --output-format csv -- python3 tools/match_pmc.py > gpurun_out/mab_${TAG}_$n.log 2>&1 || { echo "prof $n failed"; tail -5 gpurun_out/mab_${TAG}_$n.log; exit 1; }
  python3 tools/trace_summary.py gpurun_out/mab_${TAG}_$n/run_kernel_trace.csv | python3 -c "
import json,sys
d=json.load(sys.stdin); d=d if isinstance(d,list) else d.get('kernels',d)
for k in d:
    if 'match' in k['kernel']: print('$n', k['kernel'][:30], k['grid_size'], k['launches'], k['avg_us'], k['min_us'])"
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_${TAG}_$n.json 2> gpurun_out/bench_${TAG}_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_${TAG}_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$n.json')); print('$n', d['value'], 'match_2k', d['match_2k'], 'c5', d['c5_allgather_match']['batched_match_ms'], 'c1_gpu', d['c1_gpu']['ms'])"
done

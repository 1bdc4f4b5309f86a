#!/bin/bash
# Library A/B (bench lines): -m gpu suite on the working-tree build, then
# bench lines (throughput, sync single-frame latency) of ab/{nofork,fork}, twice.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_fk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fk.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for n in "$@"; do
  SIFT_HIP_LIB=ab/$n.so timeout -k 10 300 python -u bench.py --allow-ab-build --no-cpu-baseline > gpurun_out/bench_fk_${n}_$rep.json 2> gpurun_out/bench_fk_${n}_$rep.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_fk_${n}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_fk_${n}_$rep.json')); print('$n', d['value'], d['ms_per_frame'], 'sync', d['sync_ms_per_frame'], 'serial', d['single_stream']['ms_per_frame'], 'ref', json.dumps(d.get('ref_config_sync'))[:300])"
done
done
echo done

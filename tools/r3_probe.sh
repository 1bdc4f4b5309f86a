#!/bin/bash
# Round-3 probes: in-kernel clock under the batched matcher (kernel trace of the
# same run for the dispatch durations), then the single-frame/bench A/B of
# ab/NAME.so builds (tools/r3_lat.sh) and the parity tests on the first of them.
# Usage: tools/r3_probe.sh TAG "NAME1 ..."
set -o pipefail
TAG=$1; NAMES=$2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/mclk_$TAG -o run --output-format csv -- python3 tools/match_clock.py > gpurun_out/match_clock_$TAG.json 2> gpurun_out/match_clock_$TAG.err || { echo "clock failed"; tail -5 gpurun_out/match_clock_$TAG.err; exit 1; }
cat gpurun_out/match_clock_$TAG.json
python3 tools/trace_summary.py gpurun_out/mclk_$TAG/run_kernel_trace.csv | python3 -c "
import json,sys
for k in json.load(sys.stdin):
    if 'match' in k['kernel'] or 'probe' in k['kernel']: print(k['kernel'][:40], k['grid_size'], k['launches'], k['avg_us'], k['min_us'])"
[ -z "$NAMES" ] && exit 0
FIRST=default
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_$FIRST.log 2>&1
rc=$?; echo "pytest $FIRST rc=$rc"; tail -3 gpurun_out/pytest_${TAG}_$FIRST.log
[ $rc -eq 0 ] || exit $rc
bash tools/r3_lat.sh "$NAMES" $TAG

#!/bin/bash
# Round-2 GPU session: parity tests, bench, serialized per-kernel A/B of
# kernel variants (tools/ab_prof.sh, REPS interleaved repetitions), matcher
# timings per variant, rocprof kernel trace of the matcher.
# Usage: tools/r2_session.sh TAG "PROF_VARIANTS" "MATCH_VARIANTS" [REPS]
set -o pipefail
TAG=${1:-s1}
VARIANTS=${2:-}
MVARIANTS=${3:-}
REPS=${4:-1}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for v in $MVARIANTS; do
  lib=ab/$v.so; [ "$v" = default ] && lib=another-cuda-sift_amd/lib/libsift_hip.so
  SIFT_HIP_LIB=$lib timeout -k 10 120 python tools/match_time.py 2000 >> gpurun_out/match_$TAG.json 2>&1 || { echo "match_time $v failed"; tail -5 gpurun_out/match_$TAG.json; exit 1; }
done
[ -n "$MVARIANTS" ] && cat gpurun_out/match_$TAG.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mprof_$TAG -o run --output-format csv -- python3 tools/match_time.py 2000 > gpurun_out/mprof_$TAG.log 2>&1 || { echo "match prof failed"; tail -5 gpurun_out/mprof_$TAG.log; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ -n "$VARIANTS" ]; then
  names=""
  for r in $(seq 1 $REPS); do
    for v in $VARIANTS; do cp ab/$v.so ab/${v}_r$r.so; names="$names ${v}_r$r"; done
  done
  AB_BATCH=16 bash tools/ab_prof.sh $names || exit 1
  python3 tools/ab_summary.py $names > gpurun_out/ab_$TAG.txt
  cat gpurun_out/ab_$TAG.txt
fi

#!/bin/bash
# Round profile set on one GPU box (each GPU step under its own time limit,
# steps chained: a failure, fault or timeout ends the session).
#   tools/gpu_final.sh TAG pmc    -- PMC passes (tools/pmc.sh, batch 16) + matcher MFMA counters
#                                    + a roctx marker trace of the eager stages
#   tools/gpu_final.sh TAG bench  -- GPU tests, smoke, bench line, rocprof kernel stats of the bench,
#                                    the roofline pass under rocprof
# Outputs under gpurun_out/; summarise and copy into profiles/<round>/ (profiles/README.md).
set -o pipefail
TAG=${1:-final}
WHAT=${2:-bench}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$WHAT" = pmc ]; then
  bash tools/pmc.sh "$TAG" --batch 16 || exit 1
  bash tools/match_pmc.sh "$TAG" || exit 1
  timeout -k 10 120 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/marker_$TAG -o run --output-format csv -- python3 tools/profile_frames.py --frames 5 --eager > gpurun_out/marker_$TAG.log 2>&1 || { echo "marker trace failed"; tail -5 gpurun_out/marker_$TAG.log; exit 1; }
  echo "pmc session done"
  exit 0
fi
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/smoke_$TAG.txt; exit 1; }
cat gpurun_out/smoke_$TAG.txt | tail -1
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "bench prof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/roof_$TAG -o run --output-format csv -- python bench.py --roofline-only --steps 100 > gpurun_out/roof_$TAG.json 2> gpurun_out/roof_$TAG.err || { echo "roofline prof failed"; exit 1; }
echo "bench session done"

#!/bin/bash
# Round-3 profile refresh on the HEAD build: -m gpu suite, matcher sweep,
# PMC passes (16-frame batches), default bench line, rocprofv3 kernel stats of
# a bench run and of the roofline pass.  Usage: tools/r3_final.sh TAG
set -o pipefail
TAG=${1:-r3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/match_sweep.py 60 > gpurun_out/match_sweep_$TAG.json 2> gpurun_out/match_sweep_$TAG.err || { echo "match sweep failed"; tail -5 gpurun_out/match_sweep_$TAG.err; exit 1; }
tail -c 400 gpurun_out/match_sweep_$TAG.json; echo
bash tools/pmc.sh pmc_$TAG --batch 16 || exit 1
python3 tools/pmc_summary.py pmc_$TAG > gpurun_out/pmc_summary_$TAG.json || { echo "pmc summary failed"; exit 1; }
timeout -k 10 400 python -u bench.py --traffic-summary gpurun_out/pmc_summary_$TAG.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
head -c 600 gpurun_out/bench_$TAG.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/roof_$TAG -o run --output-format csv -- python3 bench.py --roofline-only --steps 100 > gpurun_out/roof_$TAG.json 2> gpurun_out/roof_$TAG.err || { echo "roofline prof failed"; tail -5 gpurun_out/roof_$TAG.err; exit 1; }
echo done

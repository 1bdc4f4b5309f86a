#!/bin/bash
# Blur staging A/B: serialized 16-frame kernel traces of each ab/NAME.so and
# alternating bench lines.
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
AB_BATCH=16 bash tools/ab_prof.sh "$@" || exit 1
python3 tools/ab_summary.py "$@" | grep -E "kernel|blur|sum of"
bash tools/r3_bench_alt.sh 2 "$@"

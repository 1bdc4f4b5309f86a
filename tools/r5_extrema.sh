#!/bin/bash
# Extrema traffic localisation (round-5 review item 1): FETCH/WRITE passes of
# the 16-frame C2 batch with one, two and three octaves (per-octave traffic by
# difference), and the outer-column-free timing variant (ab/exdiag1.so).
set -o pipefail
export TMPDIR=/tmp
for n in 1 2 3; do
  PF_ARGS="--octaves $n" AB_TAG="_o$n" tools/ab_pmc_traffic.sh ori || exit 1
done
tools/ab_pmc_traffic.sh exdiag1 || exit 1
tools/ab_prof.sh ori exdiag1 || exit 1
python3 tools/ab_summary.py ori exdiag1

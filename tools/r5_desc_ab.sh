#!/bin/bash
# Descriptor A/B (ab/dm_old.so vs ab/dm_new.so): serialized kernel durations,
# interleaved C2 throughput, descriptor-exactness test on each build.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_prof.sh ${AB_NAMES:-dm_old dm_new} || exit 1
python3 tools/ab_summary.py ${AB_NAMES:-dm_old dm_new} > gpurun_out/desc_ab_summary.txt 2>&1 || true
grep -i "descriptor" gpurun_out/desc_ab_summary.txt | head -10
bash tools/ab_run.sh ${AB_NAMES:-dm_old dm_new} || exit 1

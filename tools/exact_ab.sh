#!/bin/bash
# Exact-descriptor A/B: tools/desc_mode_bench.py with the default library and
# each ab/NAME.so given (tools/ab_variant.sh builds them).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python3 -u tools/desc_mode_bench.py --steps 30 > gpurun_out/exact_ab_default.jsonl 2>&1 || exit 1
tail -1 gpurun_out/exact_ab_default.jsonl
for V in "$@"; do
  SIFT_HIP_LIB=ab/$V.so timeout -k 10 150 python3 -u tools/desc_mode_bench.py --steps 30 > gpurun_out/exact_ab_$V.jsonl 2>&1 || exit 1
  echo "$V: $(tail -1 gpurun_out/exact_ab_$V.jsonl)"
done

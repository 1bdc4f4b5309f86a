#!/bin/bash
# Descriptor precise-math variant: flip rates vs the oracle and kernel time (A/B).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/descriptor_exact.txt
SIFT_HIP_LIB=ab/precise.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_precise.log 2>&1
rc=$?; echo "precise pytest rc=$rc"; tail -3 gpurun_out/pytest_precise.log
[ $rc -eq 0 ] || exit $rc
mv gpurun_out/descriptor_exact.txt gpurun_out/descriptor_exact_precise.txt
AB_BATCH=16 bash tools/ab_prof.sh head precise head2 precise2 || exit 1
python3 tools/ab_summary.py head precise head2 precise2 | head -6

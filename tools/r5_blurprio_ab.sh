#!/bin/bash
# s_setprio in the HBM-bound pyramid kernels (blur, extrema) under the two-stream overlap.
set -o pipefail
AB_BATCH=16 bash tools/ab_run.sh bp0 bp1 bp3 || exit 1
AB_BATCH=16 bash tools/ab_run.sh bp0 bp1 bp3 || exit 1

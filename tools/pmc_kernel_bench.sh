#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/kbpmc -o run --output-format csv -- tools/kernel_bench 20 > gpurun_out/kbpmc.log 2>&1 || { echo fail; tail -5 gpurun_out/kbpmc.log; exit 1; }
echo ok

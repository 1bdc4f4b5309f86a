#!/bin/bash
# Matcher counters: two --pmc passes (kernel trace only) over tools/match_pmc.py
# (C3 single pairs + the C5 56-pair batch), then a kernel-trace-only run.
# -> gpurun_out/mpmc_TAG_p{1,2,kt}/
set -o pipefail
TAG=${1:-m}
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/mpmc_${TAG}_p$i -o run --output-format csv -- python3 tools/match_pmc.py > gpurun_out/mpmc_${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/mpmc_${TAG}_p$i.log; exit 1; }
done
# unprofiled durations of the same kernels (kernel trace only, 400x the calls: the clock settles)
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/mpmc_${TAG}_kt -o run --output-format csv -- python3 tools/match_pmc.py 400 > gpurun_out/mpmc_${TAG}_kt.log 2>&1 || { echo "trace run failed"; tail -5 gpurun_out/mpmc_${TAG}_kt.log; exit 1; }
echo match pmc done

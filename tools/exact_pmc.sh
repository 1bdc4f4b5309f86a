#!/bin/bash
# Counters of the exact-descriptor kernel (kernel trace only, one pass per
# counter group) over tools/profile_frames.py --exact --batch 16.
# Usage: tools/exact_pmc.sh TAG  -> gpurun_out/TAG_p{1,2}/ (tools/pmc_summary.py TAG)
set -o pipefail
TAG=${1:-xpmc}
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 tools/profile_frames.py --frames 5 --batch 16 --exact > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
echo done

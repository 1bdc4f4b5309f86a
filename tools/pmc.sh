#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace) over
# tools/profile_frames.py, plus the FETCH_SIZE/WRITE_SIZE calibration binary.
# Usage: tools/pmc.sh TAG [profile_frames.py args, e.g. --batch 8]
#   -> gpurun_out/TAG_p{1..4}/, gpurun_out/TAG_calib_{fetch,write}/
set -o pipefail
TAG=${1:-pmc}
shift
PF_ARGS="$*"
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/${TAG}_p$i -o run --output-format csv -- python3 tools/profile_frames.py --frames 5 $PF_ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
if [ -x tools/hbm_calib ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_calib_$C -o run --output-format csv -- tools/hbm_calib > gpurun_out/${TAG}_calib_$C.log 2>&1 || { echo "calib $C failed"; exit 1; }
  done
fi
echo done

#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/r3_match_ab.sh m2 "new_t448 v_noepi v_nomfma" skip-tests || exit 1
for L in old new_t448; do
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  SIFT_HIP_LIB=ab/$L.so timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/mpmc_${L}_p$i -o run --output-format csv -- python3 tools/match_pmc.py > gpurun_out/mpmc_${L}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/mpmc_${L}_p$i.log; exit 1; }
done
done
echo pmc done

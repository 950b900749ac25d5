#!/bin/bash
# PMC passes over tools/exp_tile.py (all ablation modes in one process).
set -u
cd "$(dirname "$0")/.."
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc$i" -o run -- python3 tools/exp_tile.py 3000000 > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0

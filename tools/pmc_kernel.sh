#!/bin/bash
# SQ counter passes (one rocprofv3 run per set) over a diagnostic tool: TOOL=tools/x.py OUT_NAME=dir
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT_NAME:-pmck}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- python "$R/${TOOL}" >> "$OUT/pmc.log" 2>&1
  rc=$?; echo "== pass $i rc=$rc"; [ $rc -ne 0 ] && exit 1
done <<SETS
${PMC_SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS}
SETS
exit 0

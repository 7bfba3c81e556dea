#!/bin/bash
# PMC passes over tools/wgrad_check.py (B=64): per-kernel counters of the weight-gradient kernels.
#   bash tools/pmc_wgrad.sh <tag>   → gpurun_out/<tag>/p*/…; python tools/pmc_table.py gpurun_out/<tag> wgrad
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:?tag}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  B=64 timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python "$R/tools/wgrad_check.py" >> "$OUT/pmc.log" 2>&1 || exit 1
done <<SETS
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum
SETS
exit 0

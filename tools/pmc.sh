#!/bin/bash
# PMC passes for the bench workload (one rocprofv3 run per counter set; no tracing domains).
# PMC_SETS (newline-separated counter sets) overrides the default sets; OUT_NAME the output dir.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT_NAME:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  echo "== pass $i: $set" | tee -a "$OUT/pmc.log"
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS:-} >> "$OUT/pmc.log" 2>&1
  rc=$?
  echo "== pass $i rc=$rc" | tee -a "$OUT/pmc.log"
  [ $rc -ne 0 ] && exit 1
done <<SETS
${PMC_SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS}
SETS
exit 0

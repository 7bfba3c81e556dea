#!/bin/bash
# rocprofv3 kernel-trace stats + PMC passes (one run per counter set) of the bf16 bench workload.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02_bf16}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 5 ${BENCH_ARGS:---precision bf16} > "$OUT/trace.log" 2>&1 || exit 1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  echo "== pass $i: $set" >> "$OUT/pmc.log"
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS:---precision bf16} >> "$OUT/pmc.log" 2>&1
  rc=$?
  echo "== pass $i rc=$rc" >> "$OUT/pmc.log"
  [ $rc -ne 0 ] && exit 1
done <<SETS
${PMC_SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE}
SETS
exit 0

#!/bin/bash
# The training step (bench.py --mode train, B=32) by kernel: one rocprofv3 --kernel-trace --stats
# run, then one --pmc run per counter set (no tracing domains with counters), summarised by
# tools/train_pmc_table.py into gpurun_out/$TAG/${TAG}_train_kernels.json.
#   TAG=r04_train bash tools/prof_train_pmc.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?TAG}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--mode train --batch ${BATCH:-32} --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python "$R/bench.py" --steps 10 --warmup 3 $ARGS > "$OUT/trace.log" 2>&1 || exit 1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  echo "== pass $i: $set" >> "$OUT/pmc.log"
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python "$R/bench.py" --steps 2 --warmup 1 $ARGS >> "$OUT/pmc.log" 2>&1
  rc=$?
  echo "== pass $i rc=$rc" >> "$OUT/pmc.log"
  [ $rc -ne 0 ] && exit 1
done <<SETS
${PMC_SETS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS}
SETS
cd "$R"
python tools/train_pmc_table.py "$OUT" "$TAG" || exit 1
grep '^{' "$OUT/trace.log" | tail -n 1 > "$OUT/${TAG}_bench_under_trace.json" || true
exit 0

#!/bin/bash
# The committed profile of a bench workload: one rocprofv3 --kernel-trace --stats run, then one
# rocprofv3 --pmc run per counter set (no tracing domains with counters), then
# tools/pmc_summary.py → gpurun_out/$TAG/$TAG_traffic.json, next to $TAG_kernel_stats.csv (copy both
# into profiles/ to commit them; bench.py reads profiles/*_traffic.json).
#   TAG=r02_x6 PREC=x6 bash tools/profile_round.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:?TAG}
PREC=${PREC:-x6}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--no-cpu-baseline --no-bf16-leg --no-x6-leg --precision $PREC ${BENCH_ARGS:-}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
  python "$R/bench.py" --steps 20 --warmup 5 $ARGS > "$OUT/trace.log" 2>&1 || exit 1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  echo "== pass $i: $set" >> "$OUT/pmc.log"
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o pmc -- \
    python "$R/bench.py" --steps 3 --warmup 1 $ARGS >> "$OUT/pmc.log" 2>&1
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
python tools/pmc_summary.py "$OUT" "$TAG" "$PREC" ${PMC_NSB:-} || exit 1
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "$OUT/${TAG}_kernel_stats.csv"
grep '^{' "$OUT/trace.log" | tail -n 1 > "$OUT/${TAG}_bench_under_trace.json" || echo "no bench JSON line in trace.log" >&2
exit 0

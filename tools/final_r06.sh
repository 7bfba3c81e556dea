#!/bin/bash
# Round-6 measurement of one library build: the GPU test suite (-s: the printed parity numbers),
# the eval bench, the training bench three times, the Kodak-24 G9 bench, the encode/decode bench,
# and (PROFILE=1) the rocprofv3 trace + PMC summaries of the h3 and bf16 eval workloads
# (tools/profile_round.sh). Every GPU step has its own time limit; the first failure ends the call.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=${P:-r06}
O=$R/gpurun_out/final_$P
mkdir -p "$O"
cd "$R"
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$O/session.log"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$O/session.log"
  tail -n 3 "$O/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  return 0
}
if [ "${TESTS:-1}" != "0" ]; then
  step gpu_tests 700 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread -rf
fi
step bench 300 python bench.py
grep '^{' "$O/bench.log" | tail -1 > "$O/${P}_bench.json"
if [ "${BENCHES:-1}" != "0" ]; then
  for i in 1 2 3; do
    step bench_train_$i 300 python bench.py --mode train --batch 32 --no-cpu-baseline
    grep '^{' "$O/bench_train_$i.log" | tail -1 > "$O/${P}_bench_train_$i.json"
  done
  step bench_kodak 300 python bench.py --mode kodak
  grep '^{' "$O/bench_kodak.log" | tail -1 > "$O/${P}_bench_kodak_g9.json"
  step bench_encdec 300 python bench.py --mode encdec
  grep '^{' "$O/bench_encdec.log" | tail -1 > "$O/${P}_encdec_h3.json"
fi
if [ "${PROFILE:-0}" = "1" ]; then
  TAG=${P}_h3 PREC=h3 step prof_h3 900 bash tools/profile_round.sh
  TAG=${P}_bf16 PREC=bf16 step prof_bf16 900 bash tools/profile_round.sh
fi
echo done | tee -a "$O/session.log"

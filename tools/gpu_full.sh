#!/bin/bash
# Full evidence session on one GPU box: smoke, GPU tests, eval bench (+ rocprofv3 kernel stats,
# + PMC passes), train bench (+ kernel stats), Kodak mode. Every GPU step has its own time limit;
# the first failure ends the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/full
mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$O/session.log"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$O/session.log"
  tail -n 3 "$O/$name.log" | cut -c1-400
  return $rc
}
cd "$R"
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step tests 900 python -m pytest tests -m gpu -q -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
step bench 600 python bench.py || exit 1
step bench_train 600 python bench.py --mode train --batch 32 --steps 10 --warmup 3 || exit 1
step bench_kodak 600 python bench.py --mode kodak --steps 5 --warmup 2 || exit 1
step bench_2048 600 python bench.py --no-cpu-baseline --size 2048 --batch 8 --steps 10 --warmup 3 || exit 1
cd /tmp
step prof_eval 600 rocprofv3 --kernel-trace --stats -d "$O/prof_eval" -o run --output-format csv -- \
  python "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 3 || exit 1
step prof_train 600 rocprofv3 --kernel-trace --stats -d "$O/prof_train" -o run --output-format csv -- \
  python "$R/bench.py" --mode train --batch 32 --steps 5 --warmup 2 || exit 1
cd "$R"
[ "${PMC:-1}" = "1" ] && { step pmc 1200 bash tools/pmc.sh || exit 1; }
exit 0

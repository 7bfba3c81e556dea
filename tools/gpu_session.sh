#!/bin/bash
# One GPU-box session: smoke → gpu parity tests → bench (→ optional rocprofv3 stats).
# Stops at the first crash / timeout (exit status other than 0, or 1 for pytest failures).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  return $rc
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run gpu_tests 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
run bench 600 python bench.py ${BENCH_ARGS:-} || exit 1
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && run_dir=$GRAFT_REPO_ROOT/gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$run_dir" -o run --output-format csv -- \
     python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 3 \
     > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  echo "== prof rc=$?" | tee -a "$GRAFT_REPO_ROOT/gpurun_out/session.log"
fi

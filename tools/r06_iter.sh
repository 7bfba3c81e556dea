#!/bin/bash
# One GPU iteration of round 6: the GPU test suite (TESTS=0 skips, TESTSEL selects), h3 layer
# timings (tools/h3_time.py, ONLY= layers) under each of the ENVS settings ("name:VAR=val,VAR2=val"
# items; "base:" = none), and the eval bench (BENCH=0 skips). Every GPU step has its own time limit;
# a fault, abort or time-limit kill ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${OUT:-r06}
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$O/session.log"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$O/session.log"
  tail -n ${TAILN:-4} "$O/$name.log" | cut -c1-400
  case $rc in 124|134|137|139) exit $rc ;; esac
  return $rc
}
if [ "${TESTS:-1}" != "0" ]; then
  step tests 700 python -u -m pytest ${TESTSEL:-tests} -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf
fi
for e in ${ENVS:-base:}; do
  n=${e%%:*}; vars=${e#*:}
  for r in $(seq ${ROUNDS:-1}); do
    step time_${n}_$r 200 env ${vars//,/ } ONLY=${ONLY:-conv1_h3,conv2_h3,conv3_h3,deconv1_h3_int,deconv2_h3_h3out} python tools/h3_time.py
  done
done
if [ "${BENCH:-1}" != "0" ]; then
  step bench 300 python bench.py ${BENCH_ARGS:-}
fi

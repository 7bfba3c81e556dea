#!/bin/bash
# One GPU iteration: GPU tests, x6 numerics + layer timings, eval bench, and optionally an A/B of
# compile-time library variants through bench.py (VARIANTS="name:-DFLAG,-DFLAG2 name2:").
# Every GPU step has its own time limit; the first failure ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/iter
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a "$O/session.log"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$O/session.log"
  tail -n ${TAILN:-3} "$O/$name.log" | cut -c1-600
  return $rc
}
if [ "${TESTS:-1}" != "0" ]; then
  step tests 600 python -u -m pytest ${TESTSEL:-tests} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit 1
fi
[ "${X6CHECK:-1}" = "1" ] && { step x6_check 300 python tools/x6_check.py || exit 1; }
step bench 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} || exit 1
if [ -n "${VARIANTS:-}" ]; then
  for v in $VARIANTS; do
    n=${v%%:*}; f=${v#*:}; f=${f//,/ }; d=/tmp/ab_$n; mkdir -p $d
    for s in $(sed -n 's/^SRCS = //p' iclr_17_compression_amd/csrc/Makefile); do
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
        -munsafe-fp-atomics $f -c iclr_17_compression_amd/csrc/$s -o $d/${s%.hip}.o || exit 1
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libiclr17.so $d/*.o || exit 1
  done
  for r in $(seq ${ROUNDS:-2}); do
    for v in $VARIANTS; do
      n=${v%%:*}
      ICLR17_LIB=/tmp/ab_$n/libiclr17.so step ab_${n}_$r 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: v['ms'] for k, v in d.get('layers', {}).items()})" "$O/ab_${n}_$r.log" $n | tee -a "$O/ab.txt"
    done
  done
fi
exit 0

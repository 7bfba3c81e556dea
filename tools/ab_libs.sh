#!/bin/bash
# A/B of library builds on one box: the default eval bench (x6, no bf16 leg) with ICLR17_LIB set to
# each .so in turn, interleaved, R rounds. Prints value and per-layer ms per run.
#   bash tools/ab_libs.sh <outdir> <lib1.so> <lib2.so> ... (env R=3, BENCH_ARGS)
set -u
O=$(realpath -m $1); shift
mkdir -p "$O"
for r in $(seq 1 ${R:-3}); do
  for L in "$@"; do
    ICLR17_LIB=$(realpath $L) timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-bf16-leg ${BENCH_ARGS:-} 2>>"$O/err.log" | tail -1 | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $L)', d['value'], {k: v['ms'] for k, v in d['layers'].items()})" >> "$O/ab.log" || exit 1
  done
done
cat "$O/ab.log"

#!/bin/bash
# A/B of two source trees (each with its built libiclr17.so) on one box: alternating B=32
# train-step benches, 3 rounds.   bash tools/ab_train.sh <treeA> <treeB> <outdir> [bench args]
set -u
A=$(realpath $1); Bt=$(realpath $2); O=$(realpath -m $3); shift 3
mkdir -p "$O"
for r in 1 2 3; do
  for T in "$A" "$Bt"; do
    (cd "$T" && timeout -k 10 100 python -u bench.py --mode train --batch 32 --steps 30 --warmup 5 \
      --no-cpu-baseline "$@" 2>>"$O/err.log") | tail -1 | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$T', d['ms_per_step'])" >> "$O/ab.log" || exit 1
  done
done

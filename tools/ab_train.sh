#!/bin/bash
# A/B of two library builds on one box: alternating train-step benches (B=32), 3 rounds.
#   bash tools/ab_train.sh <libA.so> <libB.so> <outdir> [bench args]
set -u
A=$1; Bl=$2; O=$3; shift 3
mkdir -p "$O"
for r in 1 2 3; do
  for L in "$A" "$Bl"; do
    ICLR17_LIB=$(realpath $L) timeout -k 10 100 python -u bench.py --mode train --batch 32 --steps 30 --warmup 5 \
      --no-cpu-baseline "$@" 2>>"$O/err.log" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['ms_per_step'])" >> "$O/ab.log" || exit 1
  done
done

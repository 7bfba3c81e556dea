#!/bin/bash
# A/B(/C…) of source trees on one box: alternating tools/wgrad_check.py runs (x6 / fp32 k5 weight
# gradients at the train shapes), 3 rounds.   bash tools/ab_wgrad.sh <outdir> <tree> <tree> [...]
set -u
O=$(realpath -m $1); shift
mkdir -p "$O"
for r in 1 2 3; do
  for T0 in "$@"; do
    T=$(realpath $T0)
    echo "== $T0" >> "$O/ab.log"
    (cd "$T" && B=${B:-32} timeout -k 10 100 python -u tools/wgrad_check.py >> "$O/ab.log" 2>>"$O/err.log") || exit 1
  done
done

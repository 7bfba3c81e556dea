#!/bin/bash
# A/B of two source trees on one box: alternating default eval benches, 3 rounds.
#   bash tools/ab_eval.sh <treeA> <treeB> <outdir> [bench args]
set -u
A=$(realpath $1); Bt=$(realpath $2); O=$(realpath -m $3); shift 3
mkdir -p "$O"
for r in 1 2 3; do
  for T in "$A" "$Bt"; do
    (cd "$T" && timeout -k 10 150 python -u bench.py --no-cpu-baseline "$@" 2>>"$O/err.log") | tail -1 | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$T', d['value'], {k: v['ms'] for k, v in d['layers'].items()})" >> "$O/ab.log" || exit 1
  done
done

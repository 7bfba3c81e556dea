#!/bin/bash
# Same-box A/B of source trees (each with its built library) on the bf16 layer timings
# (tools/bf16_time.py), interleaved, 3 rounds.   bash tools/ab_bf16_trees.sh <outfile> <tree> [...]
set -u
O=$(realpath -m $1); shift
mkdir -p "$(dirname "$O")"
for r in 1 2 3; do
  for T in "$@"; do
    (cd "$T" && timeout -k 10 120 python tools/bf16_time.py --tag "$T" 2>>"$O.err") >> "$O" || exit 1
  done
done

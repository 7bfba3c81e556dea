#!/bin/bash
# Same-box A/B of the in-tree library against variant libraries (ICLR17_LIB) on the default x6
# eval bench, interleaved, 3 rounds.   bash tools/ab_x6_lib.sh <outfile> <variant.so> [...]
set -u
O=$(realpath -m $1); shift
mkdir -p "$(dirname "$O")"
for r in 1 2 3; do
  for L in intree "$@"; do
    if [ "$L" = intree ]; then
      out=$(timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-bf16-leg 2>>"$O.err") || exit 1
    else
      out=$(ICLR17_LIB=$(realpath $L) timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-bf16-leg 2>>"$O.err") || exit 1
    fi
    echo "$out" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], {k: v['ms'] for k, v in d['layers'].items()})" >> "$O" || exit 1
  done
done

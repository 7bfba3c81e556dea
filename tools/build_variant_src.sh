#!/bin/bash
# Build a variant of libiclr17.so with extra -D flags on one source of csrc/ (A/B experiments).
#   bash tools/build_variant_src.sh <source basename, e.g. wgrad_fp32> <out.so> [-DFOO=1 ...]
set -eu
SRC=$1; shift
OUT=$(realpath -m $1); shift
C=$(dirname $(realpath $0))/../iclr_17_compression_amd/csrc
T=$(mktemp -d)
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics"
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc $HF "$@" -c $C/$SRC.hip -o $T/$SRC.o
OBJS="$T/$SRC.o"
for f in engine_fp32 engine_bf16 engine_h3 aux wgrad_fp32 msssim optim datapath rans; do
  [ $f = $SRC ] || OBJS="$OBJS $C/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS
rm -rf $T

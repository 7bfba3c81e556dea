#!/bin/bash
# Build a variant of libiclr17.so with extra -D flags on engine_bf16.hip (A/B experiments).
#   bash tools/build_variant_bf16.sh <out.so> [-DFOO=1 ...]
set -eu
OUT=$(realpath -m $1); shift
C=$(dirname $(realpath $0))/../iclr_17_compression_amd/csrc
T=$(mktemp -d)
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -munsafe-fp-atomics"
/opt/rocm/bin/hipcc $HF "$@" -c $C/engine_bf16.hip -o $T/engine_bf16.o -Rpass-analysis=kernel-resource-usage 2> ${OUT%.so}.res.txt
OBJS="$T/engine_bf16.o"
for f in engine_fp32 engine_h3 aux wgrad_fp32 msssim optim datapath rans; do OBJS="$OBJS $C/$f.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $OBJS
rm -rf $T
